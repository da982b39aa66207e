set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/fps_stamps.py 2>&1 | grep -v amdgpu.ids
