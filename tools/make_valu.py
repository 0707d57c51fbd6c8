"""profiles/valu_latest.json: the VALU side of bench.py's roofline.

Inputs: a PMC summary (tools/pmc_summary.py; per-launch means of SQ_INSTS_VALU / SQ_INSTS_MFMA)
and the counting build's output (tools/exp_count.py: live wave-steps of each blend kernel over
one M1 step). Per kernel: valu_insts = SQ_INSTS_VALU - SQ_INSTS_MFMA (wave-level VALU
instructions per launch, matrix ops excluded) and evals = live wave-steps x 64 lanes, the
pixel x instance pairs the blend evaluates after the quadrant cull (every lane of a live
wave-step runs the step, predicated).

Usage: python tools/make_valu.py PMC_SUMMARY COUNT_TXT OUT [CONFIG]"""
import json
import re
import sys

pmc, cnt, dst = sys.argv[1], sys.argv[2], sys.argv[3]
config = sys.argv[4] if len(sys.argv) > 4 else "M1 P=1000000"
d = json.load(open(pmc))
text = open(cnt).read()


def grab(label):
    m = re.search(re.escape(label) + r":\s*([0-9.]+)", text)
    return int(float(m.group(1))) if m else None


def pick(prefix):
    for k, v in d.items():
        if k.startswith(prefix):
            return k, v
    return None, None  # a kernel the build no longer launches (row_sum_kernel with the atomic flush)


out = {"config": config, "source": [pmc, cnt],
       "method": "valu_insts = SQ_INSTS_VALU - SQ_INSTS_MFMA per launch (wave instructions); "
                 "evals = live wave-steps x 64 (R3DG_EXP_COUNT build, one M1 step)"}
runs = grab("m1 steps run") or 1  # the counters add up over every M1 step the counting run made
steps = {k: (v // runs if v else v) for k, v in
         {"render_fwd": grab("fwd steps done"), "render_bwd": grab("bwd live pairs")}.items()}
for name, prefix in [("render_fwd", "render_fwd_glds_kernel"), ("render_bwd", "render_bwd_glds_kernel"),
                     ("row_sum", "row_sum_kernel")]:
    k, v = pick(prefix)
    if k is None:
        continue
    ent = {"kernel": k, "valu_insts": int(round(v["SQ_INSTS_VALU"] - v.get("SQ_INSTS_MFMA", 0.0))),
           "mfma_insts": int(round(v.get("SQ_INSTS_MFMA", 0.0))), "salu_insts": int(round(v.get("SQ_INSTS_SALU", 0)))}
    if steps.get(name):
        ent["wave_steps"] = steps[name]
        ent["evals"] = steps[name] * 64
    out[name] = ent
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
