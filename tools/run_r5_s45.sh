#!/usr/bin/env bash
set -eo pipefail
bash tools/run_r5_s4.sh
bash tools/run_r5_s5.sh
