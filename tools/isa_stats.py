"""Static instruction mix of the persistent kernel's hot loop (no GPU needed).

Compiles ppls_amd/csrc/aquad.hip for gfx950 with --save-temps into a scratch directory, extracts
one k_stream instance, finds the innermost loop that holds the round (the loop whose body contains
the v_rcp_f64 of the division), and prints its instruction classes: FP64 VALU, other VALU, SALU,
LDS, branches. VGPR / SGPR / LDS usage come from the resource-usage remarks.

  python tools/isa_stats.py [--kernel _ZN2aq8k_streamILi0ELb0ELb0ELb0EEEvNS_12StreamParamsE] [-D...]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_asm(defs, out):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-c",
           "--cuda-device-only", "-S", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "ppls_amd", "csrc"),
           '-DAQ_USER_F_HEADER="%s"' % os.path.join(ROOT, "ppls_amd", "csrc", "plugins", "aq_user_gauss.h"),
           "-Rpass-analysis=kernel-resource-usage", "-o", out] + defs + [os.path.join(ROOT, "ppls_amd", "csrc", "aquad.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    return r.stderr


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_") and "_f64" in op:
        return "valu_f64"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="_ZN2aq8k_streamILi0ELb0ELb0ELb0EEEvNS_12StreamParamsE")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--dump", action="store_true", help="print the loop body")
    a = ap.parse_args()
    d = tempfile.mkdtemp()
    out = os.path.join(d, "k.s")
    remarks = compile_asm(["-D" + x for x in a.D], out)
    s = open(out).read()
    i = s.index(a.kernel + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].split("\n")
    # loops: a label line "...: ; ... Loop Header: Depth=k" and a backedge branch to it
    labels = {}
    for n, ln in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            labels[m.group(1)] = n
    best = None
    for n, ln in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", ln)
        if m and m.group(1) in labels and labels[m.group(1)] < n:
            lo, hi = labels[m.group(1)], n
            seg = body[lo:hi + 1]
            if any("v_rcp_f64" in x for x in seg) and any("v_mbcnt_lo" in x for x in seg) and any("ds_read2st64" in x for x in seg):
                if best is None or hi - lo < best[1] - best[0]:
                    best = (lo, hi)
    if best is None:
        sys.exit("no loop with v_rcp_f64 found")
    seg = [x for x in body[best[0]:best[1] + 1] if re.match(r"^\s+[a-z]", x) and not x.strip().startswith(";")]
    counts = {}
    for x in seg:
        c = classify(x.strip())
        counts[c] = counts.get(c, 0) + 1
    res = {}
    for key in ("VGPRs", "TotalSGPRs", "ScratchSize", "Occupancy", "LDS Size"):
        m = re.search(re.escape(a.kernel) + r".*?" + re.escape(key) + r"[^:]*: (\d+)", remarks, re.S)
        res[key] = m.group(1) if m else "?"
    print("kernel", a.kernel, "loop lines", best, "resources", res)
    print("instructions:", len(seg), counts, "VALU total", counts.get("valu_f64", 0) + counts.get("valu_other", 0))
    if a.dump:
        print("\n".join(body[best[0]:best[1] + 1]))


if __name__ == "__main__":
    main()
