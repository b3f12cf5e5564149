#!/bin/bash
# Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5,
# sanitizers row).  CPU only: the engine (zsummerx_amd/engine/frame.cpp) and
# the device hooks' host logic (engine/rc4_hooks_device.cpp) are built with
# -fsanitize=address,undefined against the CPU emulation of the zrc4 C-ABI
# (tests/cpp/emu_zrc4_hip.cpp), then the CPU suites that drive them run on
# those binaries: tests/test_hooks.py (reservoir levels, ring wrap, tail
# crypts, reseeds, duplicate slots) and tests/test_frame.py (wire parity with
# an oracle peer, send-queue merging, flash policy, corrupt packets, keyless
# beside keyed sessions).  Any sanitizer report aborts the binary, which fails
# its test.
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "from zsummerx_amd import build; build.build_test_tools(sanitize=True)"
export ZSX_TOOLS_BIN="$PWD/tools/bin/san"
export ZSX_STRESS="$ZSX_TOOLS_BIN/frame_stress_emu"
export ASAN_OPTIONS="abort_on_error=1:detect_leaks=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
python -m pytest tests/test_hooks.py tests/test_frame.py -m "not gpu" -q -p no:cacheprovider "$@"
# ThreadSanitizer over the reservoir's XOR worker threads (XorPool)
python -c "from zsummerx_amd import build; build.build_test_tools(sanitize='thread')"
ZSX_TOOLS_BIN="$PWD/tools/bin/tsan" TSAN_OPTIONS="halt_on_error=1" \
    python -m pytest tests/test_hooks.py -m "not gpu" -q -p no:cacheprovider -k parallel "$@"
