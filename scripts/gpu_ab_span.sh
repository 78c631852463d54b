set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=nospan,ship,span_w4,span_nopf,span_nopf_w4,span_nopf_rl,span_pf_rl,span_w4_rw3,span_w4_rw12
timeout -k 10 300 python scripts/ab_variants.py --run --variants $V --rounds 7 --launches 40 > gpurun_out/ab1_k256.json 2> gpurun_out/ab1_k256.err && \
timeout -k 10 300 python scripts/ab_variants.py --run --variants $V --rounds 7 --launches 200 --proposals 1 > gpurun_out/ab1_k1.json 2> gpurun_out/ab1_k1.err
rc=$?
python - <<'P'
import json
for f in ["gpurun_out/ab1_k256.json","gpurun_out/ab1_k1.json"]:
    try: d=json.load(open(f))
    except Exception as e: print(f, e); continue
    print(f); [print(f"  {k:14s} {v['median_us']:8.2f} us  rel {v['rel_vs_first']:.1e}") for k,v in d.items()]
P
exit $rc
