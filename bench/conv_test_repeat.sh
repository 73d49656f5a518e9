set -e
for i in 1 2 3; do
  timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread "tests/test_conv.py::test_chained_bottlenecks_grads_match_fp32" 2>&1 | tail -1
  DEDLOC_NATIVE_LIB=ab/_C_base.so timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread "tests/test_conv.py::test_chained_bottlenecks_grads_match_fp32" 2>&1 | tail -1
done
