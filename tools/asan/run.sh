#!/bin/bash
# AddressSanitizer + UBSan over the host reader (host code only; no GPU)
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/asan
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -ffp-contract=off -pthread tools/asan/reader_asan.cpp voxsrc2020_speaker_verification_amd/csrc/kaldi_host.cpp \
    -o build/asan/reader_asan
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 build/asan/reader_asan tests/golden/fm_mats.ark tests/golden/cm_mats.ark "$@"
