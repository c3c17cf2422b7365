#!/bin/bash
# Build the experiments variant of _kernels (SDML_KERNEL_EXPERIMENTS=1: timing modes, stamps, env knobs) into
# exp/_kernels_exp.so and leave the production build in the package. A GPU call swaps it in on the box only:
#   cp exp/_kernels_exp.so simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
set -e
cd "$(dirname "$0")/.."
SO=$(python -c "import sysconfig; print('simple_distributed_machine_learning_amd/_kernels' + sysconfig.get_config_var('EXT_SUFFIX'))")
rm -f "$SO.objs"
SDML_KERNEL_EXPERIMENTS=1 python -m simple_distributed_machine_learning_amd._build kernels > /tmp/build_exp.log 2>&1 || { tail -30 /tmp/build_exp.log; exit 1; }
mkdir -p exp
cp "$SO" exp/_kernels_exp.so
rm -f "$SO.objs"
python -m simple_distributed_machine_learning_amd._build kernels > /tmp/build.log 2>&1 || { tail -30 /tmp/build.log; exit 1; }
echo "exp/_kernels_exp.so and production $SO built"
