set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err || { tail -20 gpurun_out/r06a_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r06a_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('max_dpcm_lsb'), d['bitstream'].get('max_dpcm_lsb_vs_oracle'), d['host_memory'])"
timeout -k 10 900 python bench.py --gpus 4 --backend gloo > gpurun_out/r06a_rehearse4.json 2> gpurun_out/r06a_rehearse4.err || { tail -20 gpurun_out/r06a_rehearse4.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r06a_rehearse4.json').read().strip().splitlines()[-1])
print(d['value'], d['n_gpus'], d.get('max_dpcm_lsb'), d['gather'].get('parity'), d['host_memory'])"
