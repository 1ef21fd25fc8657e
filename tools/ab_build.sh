#!/bin/bash
# Build the current csrc tree into vits_amd/lib/ab_<name>.so (A/B variants of
# the kernels, compared on the GPU box in ONE call by tools/ab_conv.sh: MI355X
# boxes differ by up to ~12 % in clock, so cross-call comparisons are noise).
set -e
NAME=$1
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$R/vits_amd/csrc" EXTRA="$EXTRA" OUTDIR="$R/build/ab_$NAME" OBJDIR="$R/build/ab_obj_$NAME" >/dev/null
cp "$R/build/ab_$NAME/libvits_amd.so" "$R/vits_amd/lib/ab_$NAME.so"
echo "built vits_amd/lib/ab_$NAME.so"
