# RVQ kernel A/B: parity tests, then rocprofv3 kernel stats of tools/rvq_bench.py
set -e
mkdir -p gpurun_out/rvqx
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k rvq > gpurun_out/rvqx/test.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sh in ${RVQ_SHAPES:-5120,64,1024,8}; do
  RVQ_SHAPE=$sh RVQ_VARIANTS=${RVQ_VARIANTS:-0,2} timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rvqx/s_$sh -o r -- python -u tools/rvq_bench.py >> gpurun_out/rvqx/log.txt 2>&1
done
