#!/bin/bash
set -o pipefail
bash tools/r05_f.sh || exit $?
bash tools/r05_e.sh
