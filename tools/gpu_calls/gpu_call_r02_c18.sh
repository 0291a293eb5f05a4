set -o pipefail
TQR_FST_DTYPE=f32 timeout -k 10 200 python tools/flowstamps.py 32768 2>&1 | grep -v amdgpu.ids
