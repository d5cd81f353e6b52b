# round 5: pipelined (lnw_step_seq) A/B at the headline shape and the N=8 shard
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/seq_timing.py 65536 40 sync,seq,un2:0,un2:8,un2:15,un2:22 > gpurun_out/seq_p.log 2>&1 || { tail -20 gpurun_out/seq_p.log; exit 1; }
timeout -k 10 300 python -u tools/seq_timing.py 8192 40 sync,seq > gpurun_out/seq_p8.log 2>&1 || { tail -20 gpurun_out/seq_p8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/seq_p.log gpurun_out/seq_p8.log
