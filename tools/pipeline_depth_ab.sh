cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for rep in 1 2; do for np in 2 3 4 5; do
  NMZ_BENCH_PIPELINE=$np timeout -k 10 120 python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-secondary > /tmp/np.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/np.json'));r=d['roofline'];print('pipe', $np, 'step_ms', round(d['ms_per_step'],4), 'span_ms', round(r['kernel_ms'],4), '%.4g' % d['value'])"
done; done
