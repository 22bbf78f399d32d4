set -u
tools/ab_builds.sh "build build_prev" "--variants ALS_MFMA_WAVES=0 --rounds 5" 4
