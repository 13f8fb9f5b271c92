#!/bin/bash
# Local helper: run an arbitrary command on the GPU box with the variant libraries
# (libplba_*.so, normally gpurun-ignored) included in the snapshot.
# usage: tools/ab_cmd.sh <tag> "<command>"
cd "$(dirname "$0")/.." || exit 1
GPURUN=${GPURUN:-gpurun}  # the launcher (on PATH unless GPURUN says otherwise)
TAG=$1; CMD=$2
cp .gpurunignore /tmp/gri.abc.bak
# the tracked ignore list is restored however the run ends (error, interrupt)
trap 'cp /tmp/gri.abc.bak .gpurunignore' EXIT
grep -v "libplba_" /tmp/gri.abc.bak > .gpurunignore
"$GPURUN" --timeout 900 -- "$CMD" > /tmp/gr_abc_$TAG.log 2>&1
rc=$?
cp /tmp/gri.abc.bak .gpurunignore
tail -3 /tmp/gr_abc_$TAG.log | cut -c1-400
exit $rc
