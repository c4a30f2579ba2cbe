NAMES="base dq32 stack stackdq all32" KS=mep_attn_bwd bash scripts/r3_ab.sh || exit $?
NAMES="base" KS=mep_attn_fwd,mep_attn_bwd CFGS=cfg5 DTYPES=bf16 bash scripts/r3_ab.sh || exit $?
echo "== long (MEP_ATTN_WIDE=0) bf16:"; MEP_ATTN_WIDE=0 NAMES="base" KS=mep_attn_bwd CFGS=cfg5 DTYPES="bf16 fp32" bash scripts/r3_ab.sh || exit $?
NAMES="pvs stackdq all32" PARITY=1 KS=mep_attn_fwd CFGS=cfg3 bash scripts/r3_ab.sh || exit $?
MEP_ATTN_WIDE=0 timeout -k 10 300 python3 -m pytest tests/test_gpu_bf16.py -m gpu -q -p no:cacheprovider -k ren_cfg5 -s > gpurun_out/bf16_long.log 2>&1; echo "bf16 long rc=$?"; grep "worst\|bf16 ren" gpurun_out/bf16_long.log
