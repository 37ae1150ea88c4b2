set -o pipefail
timeout -k 10 600 python -u benchmarks/profile_predict_jobs.py --jobs vit,nbp,mmc > gpurun_out/r4_profile_predict.log 2>&1
