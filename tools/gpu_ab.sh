# A/B of library builds on the default bench (measurement): each "label|ENV=..|args" runs
# bench.py --no-cpu-baseline twice, interleaved, and prints value and E-step times.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab}; shift
mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    IFS='|' read -r label envs args <<< "$v"
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline $args > $OUT/${label}_$rep.json 2> $OUT/${label}_$rep.err || { echo "$label failed"; tail -5 $OUT/${label}_$rep.err; exit 1; }
    echo "$label#$rep: $(python -c "import json;d=json.load(open('$OUT/${label}_$rep.json'));k=d['kernel_us'];print(round(d['value']), round(k['estep'],2), round(k['estep_back_to_back'],2), round(k['m2'],2))")"
  done
done
