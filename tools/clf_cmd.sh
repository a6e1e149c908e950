export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python tools/clf_check.py --model quad13 --batch 64 > gpurun_out/clf1.json 2>&1; rc=$?; tail -5 gpurun_out/clf1.json; if [ $rc != 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/clf_check.py --model jerk --batch 64 > gpurun_out/clf2.json 2>&1; rc=$?; tail -5 gpurun_out/clf2.json; if [ $rc != 0 ]; then exit $rc; fi
timeout -k 10 180 python tools/clf_check.py --model quad13 --batch 8192 --repeats 10 > gpurun_out/clf3.json 2>&1; rc=$?; tail -3 gpurun_out/clf3.json; exit $rc
