#!/bin/bash
set -o pipefail
bash tools/r02ar_run.sh && bash tools/r02ar_ab.sh
