# Each secondary bench configuration under rocprofv3 --kernel-trace --stats (kernel
# summary + bench line per config) -> gpurun_out/$OUT/ (OUT defaults to "configs").
export TMPDIR=/tmp
o=gpurun_out/${OUT:-configs}
mkdir -p $o
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$name -o run -- python3 bench.py --no-cpu-baseline "$@" > $o/$name.json 2> $o/$name.err; }
run shard_compact --shard --force-collectives --exchange compact && run dcnv2 --model dcnv2 && run din --model din && run zipf --zipf 1.05
