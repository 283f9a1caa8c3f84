#!/bin/bash
# Build an A/B variant of liborbamd.so from this tree: lib/liborbamd_<tag>.so, objects in build_<tag>/.
# Loaded with ORBAMD_LIB_VARIANT=<tag> (orbamd/_lib.py). usage: tools/build_variant.sh <tag> [-DFLAG ...]
set -e
tag=$1; shift
cd "$(dirname "$0")/../cooperative-orb-slam_amd"
base="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable"
make -j8 OBJ=build_$tag LIB=lib/liborbamd_$tag.so HIPFLAGS="$base $*" >/dev/null
echo "built lib/liborbamd_$tag.so ($*)"
