# round-6 GPU session (one call): HEAD bench + kernel-trace profiles of the three models
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python bench.py > gpurun_out/r6/bench_head.log 2>&1 || exit 1
tail -1 gpurun_out/r6/bench_head.log
tools/prof_session.sh dn121_head || exit 1
tools/prof_session.sh vgg16_head --model vgg16 || exit 1
tools/prof_session.sh mbv2_head --model mobilenetv2 || exit 1
