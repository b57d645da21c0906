#!/usr/bin/env bash
# round 3 step 41: is the ResNet-50 FSDP step host-bound?  enqueue vs device time + cProfile; eager vs whole-step graph
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s41_host_resnet 400 python -u benchmarks/probes/host_overhead.py --layout resnet-fsdp --steps 10 --warmup 4 --cprofile 3 || exit 1
grep "\[host\]" $O/r3_s41_host_resnet.log
run r3_s41_resnet_eager 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 || exit 1
run r3_s41_resnet_graph 400 python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 --graph || exit 1
