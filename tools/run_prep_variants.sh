#!/bin/bash
# mimic_skb_prep_kernel measurement builds (tools/prep_so/*.so, built beforehand from skb.hip with the
# MIMIC_PREP_* knobs) timed alone by tools/prep_probe.py, on 1 M IMIX packets without and with the
# cfg-5 bench's 5 % header variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/prepvar; mkdir -p $D
sos=""
for n in ${PREP_SOS:-base norooms nowalk fastonly plain direct}; do sos="$sos tools/prep_so/$n.so"; done
for v in 0 0.05; do
  PREP_VARIETY=$v timeout -k 10 300 python -u tools/prep_probe.py $sos > $D/probe_v$v.log 2>&1 || { tail -20 $D/probe_v$v.log; exit 1; }
  echo "variety $v"; grep "us per launch" $D/probe_v$v.log
done
