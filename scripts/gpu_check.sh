#!/bin/bash
# GPU pass: kernel numerics, model numerics, smoke, bench, stock baseline, rocprof kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; local t=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
run kernels 900 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu
run models 600 python -m pytest tests/test_models_gpu.py -x -q -m gpu
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 10 --warmup 3
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1
  echo "prof rc=$?"
fi
