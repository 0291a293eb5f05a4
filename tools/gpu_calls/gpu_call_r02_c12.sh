set -o pipefail
timeout -k 10 60 tools/ubench/mfma_probe32 | cut -c1-300
timeout -k 10 120 python tools/debug_f32_img.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 240 python tools/order_bench.py 64 2>&1 | grep -v amdgpu.ids
