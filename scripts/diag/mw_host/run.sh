#!/bin/bash
# run.sh <merge.hip> [outdir] -- extract the multiway-merge kernels from a
# merge.hip (the shipped one, or one from history: git show REV:hpx_amd/csrc/merge.hip)
# and run them on the host under ASan + UBSan (main.cpp).  CPU only.
set -e
src=$1
out=${2:-/tmp/mw_host}
here=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$out"
# from the merge's tunables to the end of mw_stride (mw_layout and the host
# launch code stay out)
sed -n '/HPXHIP_MW_THREADS\|^constexpr int kMwThreads/,/^struct mw_layout/p' "$src" | sed '$d' > "$out/extracted.inc"
san=${MW_SAN:-address,undefined}   # MW_SAN=thread: the data-race build
g++ -std=c++20 -O1 -g -fno-omit-frame-pointer -fsanitize=$san -fno-sanitize-recover=all \
    -I"$out" -I"$here" "$here/main.cpp" -o "$out/mw_host" -lpthread
"$out/mw_host" "${@:3}"
