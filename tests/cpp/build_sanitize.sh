#!/bin/bash
# Host-only sanitizer build (reference CMakeLists.txt:67-69):
# the DwarFS frame parser of the product library and the CPU oracle, compiled
# with AddressSanitizer + UndefinedBehaviorSanitizer and driven by fuzz_host.cpp.
set -e
cd "$(dirname "$0")/../.."
mkdir -p tests/cpp/build
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
g++ -std=c++20 $SAN -Iinclude -c dwarfs_amd/csrc/ricepp_frame.cpp -o tests/cpp/build/ricepp_frame_san.o
gcc -std=c11 $SAN -c oracle/ricepp_oracle.c -o tests/cpp/build/ricepp_oracle_san.o
g++ -std=c++20 $SAN -Iinclude tests/cpp/fuzz_host.cpp tests/cpp/build/ricepp_frame_san.o \
  tests/cpp/build/ricepp_oracle_san.o -lpthread -o tests/cpp/build/fuzz_host
