set -o pipefail
# round refresh with the sustained-rate bench defaults: smoke, GPU suite, bench, rocprof + PMC
PROFILE=0 bash scripts/gpu_round.sh r61 && bash scripts/profile_round.sh r61
