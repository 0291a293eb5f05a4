set -o pipefail
timeout -k 10 300 python tools/tile_batch_check.py 2>&1 | grep -v amdgpu.ids
