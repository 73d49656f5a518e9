# round-5 session C: HIP-graph self-wait probe + the SwAV graph layout tests
mkdir -p gpurun_out
timeout -k 10 300 python bench/graph_selfwait_probe.py > gpurun_out/c_graph_probe.log 2>&1
echo "probe rc=$?"
grep -E '^case=|@@' gpurun_out/c_graph_probe.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_swav.py -k "graph" > gpurun_out/c_swav_graph_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/c_swav_graph_tests.log | tail -8
exit $rc
