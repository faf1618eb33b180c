#!/bin/bash
set -o pipefail
bash tools/archive/r02ar_run.sh && bash tools/archive/r02ar_ab.sh
