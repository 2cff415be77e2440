#!/bin/bash
# Host-sanitizer build and run of the engine (tools/host_san.c says what it drives).
#   bash tools/host_san.sh build        liblstore_ec.so with ASan + UBSan on the host code only
#                                       (each -fsanitize after -Xarch_host; the GPU code objects are
#                                       the release ones) into build/san/, and the driver beside it
#   bash tools/host_san.sh build-tsan   the same with ThreadSanitizer into build/tsan/ (run-tsan runs it)
#   bash tools/host_san.sh run [T] [I]  run the driver: the CPU part anywhere, the GPU part when a
#                                       device is visible (T threads, I calls per thread and shape)
# The GPU box runs the prebuilt build/san files (gpurun -- bash tools/host_san.sh run 8 40).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
DRV="-fsanitize=address,undefined -fno-sanitize-recover=undefined"
OUTD=build/san
if [ "${1:-}" = build-tsan ] || [ "${1:-}" = run-tsan ]; then  # ThreadSanitizer instead (host threads)
  SAN="-Xarch_host -fsanitize=thread"
  DRV="-fsanitize=thread"
  OUTD=build/tsan
fi
case "${1:-run}" in
build|build-tsan)
  mkdir -p $OUTD
  make -s -j8 -C lstore_amd/csrc ../../$OUTD/liblstore_ec.so OUT=../../$OUTD/liblstore_ec.so \
    OBJDIR=../../$OUTD/obj EXTRA="-g -fno-omit-frame-pointer $SAN" || exit 1
  # compiled as C, linked by clang++ so that the sanitizer's C++ runtime (operator new / delete,
  # the function-local static guards the library's C++ uses) is the one in the process
  /opt/rocm/llvm/bin/clang -std=c11 -O1 -g -fno-omit-frame-pointer $DRV -Wall -c -o $OUTD/host_san.o tools/host_san.c \
    -Iinclude || exit 1
  /opt/rocm/llvm/bin/clang++ $DRV -o $OUTD/host_san $OUTD/host_san.o -L$OUTD -llstore_ec -Wl,-rpath,'$ORIGIN' \
    -lpthread || exit 1
  echo "built $OUTD/host_san"
  ;;
run-tsan)
  export TSAN_OPTIONS="halt_on_error=${TSAN_HALT:-1}:second_deadlock_stack=1"
  export LSEC_JITC="$PWD/lstore_amd/lsec_jitc"
  timeout -k 10 "${HOST_SAN_TIMEOUT:-600}" $OUTD/host_san "${2:-4}" "${3:-40}"
  ;;
run)
  mkdir -p gpurun_out
  # leaks: the HIP runtime keeps allocations to process exit; the driver's own are checked
  export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_stack_use_after_return=1:strict_string_checks=1"
  export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
  export LSEC_JITC="$PWD/lstore_amd/lsec_jitc"
  timeout -k 10 "${HOST_SAN_TIMEOUT:-600}" build/san/host_san "${2:-4}" "${3:-40}"
  ;;
*)
  echo "usage: $0 build | run [threads] [iters]" >&2
  exit 2
  ;;
esac
