#!/bin/bash
# round 4 close, part 2: rocprofv3 trace + PMC passes of the bench's own command, C2..C5
# (profiles/current_c<config>.json = each bench line's traffic source)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for c in ${@:-2 3 4 5}; do bash scripts/gpu_prof.sh round4b_c$c $c || exit $?; done
