cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in 1 0; do
  MIMIC_JIT_SKBFAST=$v CFG=skb NAME=skb_fast$v TAG=r05c REQ=1 SQ=1 timeout -k 10 600 bash tools/profile.sh || { echo "profile $v failed"; tail -20 gpurun_out/prof_r05c/*.log; exit 1; }
  tail -1 gpurun_out/prof_r05c/summary_skb_fast$v.log | cut -c1-1500
done
