set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04d/cfg
timeout -k 10 500 python -u bench.py --no-cpu-baseline --K 30 --P 50000 --E 10000000 --test-frac 0 --steps 10 --warmup 2 --roofline-launches 5 > gpurun_out/r04d/cfg/k30_10m.json 2> gpurun_out/r04d/cfg/k30_10m.err || { tail -20 gpurun_out/r04d/cfg/k30_10m.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04d/cfg/k30_10m.json')); print(round(d['value'],1), d['iteration']['us'], d['config']['E_train'], {k: round(v['back_to_back'],1) for k, v in d['kernel_us'].items()})"
bash tools/gpu_r04_prof.sh r04d/prof20 gpurun_out/r04d/pmc_r04_K20.json 200 10 --K 20 --samples 8 && \
bash tools/gpu_r04_prof.sh r04d/prof30 gpurun_out/r04d/pmc_r04_K30.json 30 4 --K 30 --P 50000 --E 10000000 --test-frac 0
