#!/bin/bash
set -o pipefail
PART=prof bash tools/r03i_run.sh && bash tools/r03j_unesc_ab.sh
