set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 300 python -u -m pytest tests/test_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1 || { tail -40 gpurun_out/g1/pytest.log; exit 1; }
tail -3 gpurun_out/g1/pytest.log
for B in 256 32; do
for G in "" "--cuda-graph"; do
timeout -k 10 200 python -u examples/resnet_benchmark.py --arch resnet50 --use-fsdp --amp --channels-last --batch-size $B --epochs 3 --steps-syn 20 $G --json-out gpurun_out/g1/r50_b${B}${G:+_graph}.json > gpurun_out/g1/r50_b${B}${G:+_graph}.log 2>&1 || { tail -30 gpurun_out/g1/r50_b${B}${G:+_graph}.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/g1/r50_b${B}${G:+_graph}.json'));print('B=$B graph=$G', round(d['images_per_sec'],1), d['final_loss'])"
done; done
