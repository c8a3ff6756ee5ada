# Timing-only A/B (results of _xor are wrong for subtracting streams; never
# shipped): the XSL xor as VOP2 v_xor_b32_e32 (sign mask dropped) vs the
# product's VOP3 v_bitop3 with the sign mask -- does a VOP2 form issue
# cheaper than a VOP3 one at the kernel's 2 waves per SIMD?
set -o pipefail
export TMPDIR=/tmp
bash tools/debug/ab_variants.sh ab_xor "base _xor" 8:1,8:2,8:8 4 > gpurun_out/ab_xor.log 2>&1 || { tail gpurun_out/ab_xor.log; exit 1; }
python tools/debug/ab_summary.py gpurun_out/ab_xor/kb.jsonl 2>&1 | tail -8
