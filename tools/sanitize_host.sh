#!/bin/bash
# Host-code sanitizer builds. GPU sanitizers are not used: kernels are checked with
# host twins + numerics tests; the host C++ (regex compiler, batch packer threads) runs here under
# ASan+UBSan and TSan. Usage: tools/sanitize_host.sh [iterations]
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p build/sanitize
SRC="tools/native/selftest.cpp csrc/regex/jregex.cpp csrc/io/docs.cpp csrc/io/json_in.cpp csrc/io/http_server.cpp"
CXX=${CXX:-g++}
$CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -pthread -Icsrc $SRC -o build/sanitize/selftest_asan
$CXX -std=c++17 -O1 -g -fsanitize=thread -pthread -Icsrc $SRC -o build/sanitize/selftest_tsan
ASAN_OPTIONS=detect_leaks=1 ./build/sanitize/selftest_asan "${1:-3000}"
TSAN_OPTIONS=halt_on_error=1 ./build/sanitize/selftest_tsan 300
