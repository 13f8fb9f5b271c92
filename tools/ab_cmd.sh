#!/bin/bash
# Local helper: run an arbitrary command on the GPU box with the variant libraries
# (libplba_*.so, normally gpurun-ignored) included in the snapshot.
# usage: tools/ab_cmd.sh <tag> "<command>"
cd /root/repo || exit 1
TAG=$1; CMD=$2
cp .gpurunignore /tmp/gri.abc.bak
grep -v "libplba_" /tmp/gri.abc.bak > .gpurunignore
/usr/local/graft/bin/gpurun --timeout 900 -- "$CMD" > /tmp/gr_abc_$TAG.log 2>&1
rc=$?
cp /tmp/gri.abc.bak .gpurunignore
tail -3 /tmp/gr_abc_$TAG.log | cut -c1-400
exit $rc
