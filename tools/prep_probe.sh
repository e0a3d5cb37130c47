#!/bin/bash
# mimic_skb_prep_kernel alone (tools/prep_probe.py): builds skb.hip as a small shared library (once;
# VARIANTS="name:-DFLAG ..." adds measurement builds, e.g. "plain:-DMIMIC_PREP_PLAIN"), then times it
# with and without the record output
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/prep; mkdir -p $D tools/prep_so
sos=""
for v in base: $VARIANTS; do
  n=${v%%:*}; f=${v#*:}
  [ -f tools/prep_so/$n.so ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value $f \
      mimic_amd/csrc/skb.hip -o tools/prep_so/$n.so || exit 1
  sos="$sos tools/prep_so/$n.so"
done
timeout -k 10 300 python -u tools/prep_probe.py $sos > $D/probe.log 2>&1; rc=$?
tail -6 $D/probe.log; exit $rc
