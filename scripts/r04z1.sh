#!/bin/bash
# Round 4 closing session, part 1: smoke, the whole GPU suite, the default
# bench line and its rocprof kernel statistics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04z}
bash scripts/r03_session.sh $T smoke tests bench prof
