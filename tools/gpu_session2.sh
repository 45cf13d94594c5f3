#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_mpi_layer.py -m gpu -q > gpurun_out/mpi_tests.log 2>&1; rc=$?
echo "mpi tests rc=$rc"; tail -8 gpurun_out/mpi_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/rccl_probe.py > gpurun_out/probe.log 2>&1; rc=$?
echo "probe rc=$rc"; grep PROBE gpurun_out/probe.log; tail -4 gpurun_out/probe.log
case $rc in 0|1) ;; *) exit $rc;; esac
B="python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/traffic_node_r8_16mib_float.json node_r8_16mib_float
ls gpurun_out/pmc_fetch/* | head
exit 0
