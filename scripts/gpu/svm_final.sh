# final SVM numbers: solver timings and whole-fit comparison with sklearn
set -o pipefail
timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/f_svm.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 8192 > gpurun_out/f_vsref.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 32768 >> gpurun_out/f_vsref.log 2>&1
