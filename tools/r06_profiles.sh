#!/bin/bash
# Round 6: rocprofv3 evidence for C2, C3 and C4 on this tree's library, one
# profile_round.sh per config (plain bench line, kernel trace, PMC passes), so
# that profiles/pmc_traffic.json can cite digest-tied traffic for all three.
set -o pipefail
bash tools/profile_round.sh c2_r06 && echo "== c2 ok" &&
bash tools/profile_round.sh c3_r06 --file-gib 64 --no-e2e --no-cpu-baseline --no-other-configs && echo "== c3 ok" &&
bash tools/profile_round.sh c4_r06 --config c4 --no-e2e --no-cpu-baseline --no-other-configs && echo "== c4 ok"
