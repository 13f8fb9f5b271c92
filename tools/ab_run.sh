#!/bin/bash
# Local helper: send the variant libraries (normally gpurun-ignored) with one gpurun call.
# usage: tools/ab_run.sh <tag> "<cfg list>" <lib> [<lib> ...]
cd /root/repo || exit 1
TAG=$1; CFGS=$2; shift 2
cp .gpurunignore /tmp/gri.ab.bak
grep -v "libplba_" /tmp/gri.ab.bak > .gpurunignore
echo './pl-slam-plucker_amd/libplba_stamps.so' >> .gpurunignore
CMD=""
for c in $CFGS; do CMD="$CMD bash tools/gpu_variants.sh $TAG $c $* &&"; done
/usr/local/graft/bin/gpurun --timeout 900 -- "${CMD} true" > /tmp/gr_ab_$TAG.log 2>&1
rc=$?
cp /tmp/gri.ab.bak .gpurunignore
tail -1 /tmp/gr_ab_$TAG.log
exit $rc
