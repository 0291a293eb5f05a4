set -o pipefail
PASS=lds bash tools/pmc_stall.sh
