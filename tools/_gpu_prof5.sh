#!/bin/bash
# end-of-round cfg2 profiles: kernel trace (20 timed steps, markers) and the PMC passes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile.sh r05p trace pmc
ls gpurun_out/r05p
