set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wu
for w in 5 25 45 65 85; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup $w > gpurun_out/wu/w$w.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/wu/w$w.log').read().strip().splitlines()[-1]); print('warmup $w steps 20', round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],4))"
done
