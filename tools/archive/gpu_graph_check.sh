set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/graph_memset_probe.py > gpurun_out/memset.log 2>&1; echo memset=$?
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_graph.py > gpurun_out/t_graph.log 2>&1; echo tgraph=$?
for w in newcrf guidedepth; do for a in bf16 fp32; do
timeout -k 10 300 python -u tools/graph_check.py $w $a 6 >> gpurun_out/graph_check.log 2>&1; echo check_${w}_${a}=$?
done; done
