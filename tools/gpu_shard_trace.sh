# The row-sharded step at world 1 (RCCL forced, compact and slot exchanges) under
# rocprofv3 --kernel-trace --stats -> gpurun_out/$OUT/
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r5f}
mkdir -p $o
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$name -o run -- python3 bench.py --no-cpu-baseline --no-h2d "$@" > $o/$name.json 2> $o/$name.err || { tail -5 $o/$name.err; exit 1; }; python3 -c "import json; d=json.load(open('$o/$name.json')); print('$name', d['ms_per_step'])"; }
run shard_compact --shard --force-collectives --exchange compact && run shard_slot --shard --force-collectives --exchange slot
