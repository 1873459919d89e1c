#!/bin/bash
# Builds the C++ facade test against the product library and the CPU oracle.
set -e
cd "$(dirname "$0")/../.."
mkdir -p tests/cpp/build
hipcc -O2 -std=c++20 -Iinclude -o tests/cpp/build/facade_test tests/cpp/facade_test.cpp \
  -Ldwarfs_amd/lib -lricepp_amd -Loracle/build -lricepp_oracle -lflac_oracle \
  -Wl,-rpath,'$ORIGIN/../../../dwarfs_amd/lib' -Wl,-rpath,'$ORIGIN/../../../oracle/build'
