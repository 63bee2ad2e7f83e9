# Selected GPU tests (GPU box): TESTS="tests/a.py tests/b.py" bash tools/run_tests_sel.sh
set -o pipefail
O=gpurun_out/${TAG:-sel}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && grep -E "^E |FAILED|Error" $O/tests.log | head -40
exit $rc
