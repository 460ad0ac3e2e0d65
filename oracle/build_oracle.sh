#!/usr/bin/env bash
# oracle/build_oracle.sh -- TEST INFRASTRUCTURE ONLY: builds the C restatement.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
mkdir -p "$HERE/_build"
gcc -O3 -std=c11 -fPIC -shared -o "$HERE/_build/liboracle.so" "$HERE/crc32c_oracle.c" -lpthread
echo "built $HERE/_build/liboracle.so"
