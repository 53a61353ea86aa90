cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for cfg in "20 3" "100 3" "20 4" "100 4" "20 2" "20 3" "100 3"; do set -- $cfg
  NMZ_BENCH_PIPELINE=$2 timeout -k 10 120 python3 $R/bench.py --steps $1 --warmup 3 --no-cpu-baseline --no-secondary > /tmp/sv.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/sv.json'));print('steps=$1 NP=$2', 'step_ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4), '%.4g' % d['value'])"
done
