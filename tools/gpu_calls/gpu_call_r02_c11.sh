set -o pipefail
timeout -k 10 60 tools/ubench/mfma_probe32 | cut -c1-400
