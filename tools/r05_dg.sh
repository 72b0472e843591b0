#!/bin/bash
set -o pipefail
bash tools/r05_g.sh || exit $?
bash tools/r05_d.sh
