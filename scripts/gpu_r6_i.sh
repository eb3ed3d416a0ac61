#!/bin/bash
# r6i: halo conv timing probe (full / no MFMA / no read-out / neither)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for d in 0 1 2 3; do DL4J_AMD_HALO_DBG=$d timeout -k 10 120 python3 tools/halo_probe.py || exit 1; done
for d in 0 1 2 3; do DL4J_AMD_HALO_DBG=$d timeout -k 10 120 python3 tools/halo_probe.py --hw 56 --batch 256 || exit 1; done
