#!/bin/bash
# Build the library of git revision $1 as variant $2 (libgicp_hip_$2.so, GICP_LIB_VARIANT=$2) for A/B timing.
set -e
rev=$1; name=$2; root=$(git rev-parse --show-toplevel); tmp=/tmp/rev_$name
rm -rf "$tmp"; mkdir -p "$tmp"
git -C "$root" archive "$rev" generalized-icp_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/generalized-icp_amd/csrc" -j4 VARIANT="$name" OUT="$root/generalized-icp_amd/gicp/libgicp_hip_$name.so"
