set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/fix_tests.log python -u -m pytest tests/kernels/test_convnet_gpu.py -x -v --timeout 120 --timeout-method thread -k "fix or in_launch" || exit 1
grep -q " failed\| error" gpurun_out/fix_tests.log && exit 1
$S 400 gpurun_out/fix_ab.log scripts/ab_env.sh DISTLEARN_FIX "0 1 2" 4 || exit 1
cat gpurun_out/fix_ab.log
DISTLEARN_FIX=2 $S 240 gpurun_out/fix_prof.log rocprofv3 --kernel-trace -d gpurun_out/prof_fix -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof_fix/run_results.db > gpurun_out/timeline_fix.txt 2>&1
cat gpurun_out/timeline_fix.txt
