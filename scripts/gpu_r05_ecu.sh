# Round 5: EdgeConv gather batching (backward: 16 slot rows in flight per lane; forward: 8 neighbours per batch): tests, then the
# DGCNN step A/B: ecu4 = four-slot gather rounds (-DPCS_AB_EC_U=4), ecold = that and one forward neighbour at a time (-DPCS_AB_EC_FB=1), as in round 4.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_ecu; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_edgeconv.py tests/test_gpu_models.py -k "edgeconv or dgcnn or EdgeConv" -x -q -p no:cacheprovider --timeout 800 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_libs_ab.sh r05_ab18 3 "- _ecu4 _ecold" --model dgcnn
