#!/bin/bash
# GPU kernel numerics run (used with gpurun). Writes logs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.get_device_name(0))"
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider "$@" > gpurun_out/kernels.log 2>&1
rc=$?
echo "pytest exit $rc"
tail -40 gpurun_out/kernels.log
exit $rc
