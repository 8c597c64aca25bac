set -o pipefail
mkdir -p gpurun_out/r5/a
O=gpurun_out/r5/a
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bench.py "tests/test_gpu.py::test_ipc_event_domains_in_sequence_and_host_run_ahead" "tests/test_gpu.py::test_colocated_completion_switching_two_ranks" "tests/test_gpu.py::test_colocated_caller_stream_two_ranks" "tests/test_gpu.py::test_device_exchange" -k "not PeerCopyEngine" > $O/pytest.log 2>&1 &&
timeout -k 10 200 python bench.py > $O/bench1.json 2> $O/bench1.err &&
timeout -k 10 300 python bench.py --gpus 2 > $O/bench2.json 2> $O/bench2.err
