set -o pipefail
timeout -k 10 120 python tools/debug_f32.py 2>&1 | grep -v amdgpu.ids
