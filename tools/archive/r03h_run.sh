#!/bin/bash
# Round 3: long4 A/B (tools/r03g_ab.sh), then tools/r03f_run.sh (new GPU tests + N>1 rehearsals).
set -o pipefail
bash tools/r03g_ab.sh && bash tools/r03f_run.sh
