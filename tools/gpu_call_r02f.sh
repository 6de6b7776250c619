# r02: rocprof evidence (kernel stats + FETCH/WRITE passes) for the C2 kernel and the n = 8 fold
set -o pipefail
bash tools/profile_local.sh r02 > gpurun_out/prof_local_r02.log 2>&1 && \
bash tools/profile_fold.sh r02 8 > gpurun_out/prof_fold_r02.log 2>&1
