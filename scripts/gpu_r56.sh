set -o pipefail
# Re-entry verification of the current tree: smoke, full GPU suite, bench, rocprof + PMC.
bash scripts/gpu_round.sh r56 && bash scripts/profile_round.sh r56
