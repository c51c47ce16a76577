#!/bin/bash
# The CPU suite (pytest -m "not gpu") against AddressSanitizer + UndefinedBehaviorSanitizer builds of the
# host library (chiaroscuro-raytracer_amd/san/lib: the .rtc parser, OBJ/MTL/PNG loader, EXR codec,
# checkpoint/resume, kd build, RayTracer, preview session) and of the oracle (oracle/_san), SURVEY §5.
# The sanitizer runtimes are preloaded into the (uninstrumented) Python; leak checking is off (the
# interpreter and the HIP runtime keep allocations to exit), every other report aborts the run.
#   scripts/sanitize_cpu_suite.sh [pytest args...]     (log: profiles/r06_sanitize_cpu_suite.txt)
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C chiaroscuro-raytracer_amd -j8
make -s -C chiaroscuro-raytracer_amd SANITIZE=1 -j8
make -s -C oracle all san
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0:allocator_may_return_null=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
export CHIARO_LIB_DIR="$PWD/chiaroscuro-raytracer_amd/san/lib"
export CHIARO_ORACLE_DIR="$PWD/oracle/_san"
python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@"
