set -o pipefail
mkdir -p gpurun_out/dw
timeout -k 10 120 ./tools/micro/dmapat > gpurun_out/dw/dmapat.json 2> gpurun_out/dw/dmapat.err || { cat gpurun_out/dw/dmapat.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/dw/dmapat.json'))
for r in d['runs']: print(r)"
