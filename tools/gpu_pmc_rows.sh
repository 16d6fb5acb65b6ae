#!/bin/bash
# PMC passes on the build kernels (both variants) at p = 50.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
CMPC_BUILD_VARIANT=rows bash tools/pmc_build.sh pr 50 || exit $?
CMPC_BUILD_VARIANT=wave bash tools/pmc_build.sh pw 50 || exit $?
python tools/pmc_print.py pr; python tools/pmc_print.py pw
