#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_session13.sh &&
bash tools/r4_session14.sh
