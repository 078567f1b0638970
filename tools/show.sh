# summarise bench JSON lines of a gpurun_out tag
for f in gpurun_out/$1/bench*.json; do
python - "$f" <<'PY'
import json,sys
f=sys.argv[1]
try:
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print("%-40s %9.0f it/s  %7.2f us/it  %s  frac=%.3f" % (f.split('/')[-1], d['value'], d['ms_per_step']*1e3, {k: round(v,2) for k,v in d['kernel_us'].items()}, d['roofline']['frac']))
except Exception as e:
    print(f, "ERR", e)
PY
done
