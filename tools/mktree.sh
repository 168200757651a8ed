#!/bin/bash
# Scratch build tree of the HIP library (A/B experiments on the GPU box):
#   [GEN_BLOCK=n] tools/mktree.sh <dir> <patches|-> [extra hipcc flags...]
# copies the Python package and csrc/, applies the comma-separated patches in
# order (*.py: run as `python3 script <dir>`, else `patch -p1`) and builds
# <dir>/trajopt-1_amd/lib/libtrajopt_hip.so with the extra flags appended.
set -e
cd "$(dirname "$0")/.."
d=$1; p=$2; shift 2
rm -rf "$d"; mkdir -p "$d/trajopt-1_amd" "$d/include"
cp -r trajopt-1_amd/trajopt_amd trajopt-1_amd/csrc "$d/trajopt-1_amd/"
cp include/*.h "$d/include/"
rm -rf "$d/trajopt-1_amd/trajopt_amd/__pycache__"
if [ "$p" != "-" ]; then
  IFS=',' read -ra PS <<< "$p"
  for q in "${PS[@]}"; do
    case "$q" in
      *.py) python3 "$q" "$d" ;;
      *) patch -s -d "$d" -p1 < "$q" ;;
    esac
  done
fi
make -s -C "$d/trajopt-1_amd/csrc" -j8 EXTRA="$*" ${GEN_BLOCK:+GEN_BLOCK=$GEN_BLOCK}
