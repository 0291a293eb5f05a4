set -o pipefail
bash tools/pmc_stall.sh
