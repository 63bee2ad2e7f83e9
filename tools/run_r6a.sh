# Round 6, call A (GPU box): frame tests, cfg5 A/B (r5 lib, product, Kafka at
# 4 waves), Kafka traffic calibration with FETCH_SIZE and raw TCC counters.
set -o pipefail
O=gpurun_out/r6a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py -x -v --timeout 120 --timeout-method thread > $O/frame_tests.log 2>&1; rc=$?
tail -3 $O/frame_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/frame_tests.log | head -20; exit 1; }
TAG=r6a/ab LIBS="r5 prod kw4" bash tools/ab_libs.sh || exit 2
timeout -k 10 200 python -u tools/calib_kafka.py > $O/calib.log 2>&1 || { tail -20 $O/calib.log; exit 3; }
cat $O/calib.log
i=0
for c in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/calib_pmc$i -o pmc --output-format csv -- python3 -u tools/calib_kafka.py > $O/calib_pmc$i.log 2>&1 || { tail -5 $O/calib_pmc$i.log; exit 4; }
  echo pmc $i done
done
python3 tools/pmc_dispatches.py $O/calib_pmc1 $O/calib_pmc2 $O/calib_pmc3 > $O/calib_pmc_summary.txt 2>&1
grep -v "elementwise" $O/calib_pmc_summary.txt | head -90
