#!/bin/bash
# Local helper: send the variant libraries (normally gpurun-ignored) with one gpurun call.
# usage: tools/ab_run.sh <tag> "<cfg list>" <lib> [<lib> ...]
cd "$(dirname "$0")/.." || exit 1
GPURUN=${GPURUN:-gpurun}  # the launcher (on PATH unless GPURUN says otherwise)
TAG=$1; CFGS=$2; shift 2
cp .gpurunignore /tmp/gri.ab.bak
# the tracked ignore list is restored however the run ends (error, interrupt)
trap 'cp /tmp/gri.ab.bak .gpurunignore' EXIT
grep -v "libplba_" /tmp/gri.ab.bak > .gpurunignore
echo './pl-slam-plucker_amd/libplba_stamps.so' >> .gpurunignore
CMD=""
for c in $CFGS; do CMD="$CMD bash tools/gpu_variants.sh $TAG $c $* &&"; done
"$GPURUN" --timeout 900 -- "${CMD} true" > /tmp/gr_ab_$TAG.log 2>&1
rc=$?
cp /tmp/gri.ab.bak .gpurunignore
tail -1 /tmp/gr_ab_$TAG.log
exit $rc
