#!/usr/bin/env bash
# The CPU oracle (oracle/mvs_oracle.c) under AddressSanitizer + UBSan (host
# only; container or GPU-box host): the oracle's CPU tests and golden checks
# against oracle/_build/liboracle_asan.so.  Any report fails the run.
set -eu
cd "$(dirname "$0")/.."
make -s -C oracle asan
export MVS_ORACLE_LIB=$PWD/oracle/_build/liboracle_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-4}
LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so) \
  python3 -m pytest -x -q -p no:cacheprovider -m "not gpu" tests/test_oracle_cpu.py tests/test_golden.py tests/test_ref_fixtures.py "$@"
