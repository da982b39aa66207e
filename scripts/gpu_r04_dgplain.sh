# DMA dgrad over a plain (materialised) dZ operand: bitwise tests, isolated A/B, PointNet++ step
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/dgplain; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dgrad_dma.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
rm -f $out/ab.log
for d in 1; do for m in plain; do
  PCS_DGRAD_DMA=$d PCS_DGRAD_MODE=$m timeout -k 10 120 python -u scripts/dgrad_ab.py >> $out/ab.log 2>&1 || exit 1
done; done
grep dma= $out/ab.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --secondary none --no-cpu-baseline --no-drop-in > $out/b$i.json 2>$out/b$i.err || { tail -5 $out/b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], [ (t['kernel'], t['in_step_ms']) for t in r['top_kernels'] if 'dgrad' in t['kernel'] or 'gemm_rows' in t['kernel']])" $out/b$i.json
done
