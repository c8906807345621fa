"""Static instruction mix of the persistent kernel's hot loop (no GPU needed).

Compiles ppls_amd/csrc/aquad.hip for gfx950 with --save-temps into a scratch directory, extracts
one k_stream instance, finds the innermost loop that holds the round (the loop whose body contains
the v_rcp_f64 of the division), and prints its instruction classes: FP64 VALU, other VALU, SALU,
LDS, branches. VGPR / SGPR / LDS usage come from the resource-usage remarks.

  python tools/isa_stats.py [--kernel _ZN2aq8k_streamILi0ELb0ELb0ELb0ELi12ELb0EEEvNS_12StreamParamsE] [-D...]
  python tools/isa_stats.py --sizes [-D...]     # code bytes of every k_stream instance (device object)
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_asm(defs, out):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-c", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
           "--cuda-device-only", "-S", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "ppls_amd", "csrc"),
           '-DAQ_USER_F_HEADER="%s"' % os.path.join(ROOT, "ppls_amd", "csrc", "plugins", "aq_user_gauss.h"),
           "-Rpass-analysis=kernel-resource-usage", "-o", out] + defs + [os.path.join(ROOT, "ppls_amd", "csrc", "aquad.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    return r.stderr


def code_sizes(defs):
    """Machine-code bytes of every k_stream instance: a device-only object, its symbol sizes."""
    d = tempfile.mkdtemp()
    obj = os.path.join(d, "k.o")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-c",
           "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "--cuda-device-only", "--no-gpu-bundle-output", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "ppls_amd", "csrc"),
           '-DAQ_USER_F_HEADER="%s"' % os.path.join(ROOT, "ppls_amd", "csrc", "plugins", "aq_user_gauss.h"),
           "-o", obj] + defs + [os.path.join(ROOT, "ppls_amd", "csrc", "aquad.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    sym = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-sW", "--demangle", obj], capture_output=True,
                         text=True, check=True).stdout
    out = {}
    for ln in sym.splitlines():
        f = ln.split(None, 7)   # Num: Value Size Type Bind Vis Ndx Name
        if len(f) == 8 and f[3] == "FUNC" and "k_stream" in f[7] and not f[7].endswith("(.kd)"):
            out[f[7]] = int(f[2])
    return out


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
    ap.add_argument("--kernel", default="_ZN2aq8k_streamILi0ELb0ELb0ELb0ELi12ELb0EEEvNS_12StreamParamsE")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--mllvm", action="append", default=[], help="an LLVM option (e.g. -amdgpu-sched-strategy=max-ilp)")
    ap.add_argument("--dump", action="store_true", help="print the loop body")
    ap.add_argument("--first-backedge", action="store_true",
                    help="bottom-tested loop: count up to the first conditional back-edge")
    ap.add_argument("--keep", help="also write the kernel's assembly (with labels) to this file")
    ap.add_argument("--sizes", action="store_true", help="print the code bytes of every k_stream instance")
    a = ap.parse_args()
    if a.sizes:
        sz = code_sizes(["-D" + x for x in a.D])
        for k in sorted(sz):
            print("%7d B  %s" % (sz[k], k))
        return
    d = tempfile.mkdtemp()
    out = os.path.join(d, "k.s")
    remarks = compile_asm(["-D" + x for x in a.D] + [y for m in a.mllvm for y in ("-mllvm", m)], out)
    s = open(out).read()
    i = s.index(a.kernel + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].split("\n")
    if a.keep:
        open(a.keep, "w").write(s[i:j])
    # blocks: a label line ".LBBx_y:" with LLVM's loop comment ("Loop Header: Depth=k" or "in Loop:
    # Header=BBx_z Depth=k"); the round's loop is the innermost loop whose blocks hold the v_rcp_f64 of
    # the division, a v_mbcnt_lo and a ds_read2st64 -- counted over ALL its blocks (a rotated loop
    # places some of them after its back-edge)
    blocks = []   # (label, header_of_loop_or_None, depth, lines)
    cur = None
    for ln in body:
        m = re.match(r"^(\.LBB(\d+_\d+)):(.*)$", ln)
        if m:
            hdr, depth = None, 0
            mh = re.search(r"Loop Header: Depth=(\d+)", m.group(3))
            mi = re.search(r"in Loop: Header=BB(\d+_\d+) Depth=(\d+)", m.group(3))
            if mh:
                hdr, depth = m.group(2), int(mh.group(1))
            elif mi:
                hdr, depth = mi.group(1), int(mi.group(2))
            cur = [m.group(1), hdr, depth, []]
            blocks.append(cur)
        elif cur is not None:
            mh = re.search(r"Loop Header: Depth=(\d+)", ln)
            if mh and ln.strip().startswith(";") and not any(x.strip() and not x.strip().startswith(";") for x in cur[3]):
                cur[1], cur[2] = cur[0][4:], int(mh.group(1))   # "; => This Inner Loop Header" under the label
            cur[3].append(ln)
    inloop = lambda b, key: b[1] == key[0] and b[2] >= key[1]
    keys = {(b[1], b[2]) for b in blocks if b[1]}
    best = None
    for key in keys:
        lines = [x for b in blocks if inloop(b, key) for x in b[3]]
        if any("v_rcp_f64" in x for x in lines) and any("v_mbcnt_lo" in x for x in lines) and any("st64" in x for x in lines):
            if best is None or key[1] > best[1]:
                best = key
    if best is None:
        sys.exit("no loop with v_rcp_f64 found")
    # the hot path: the contiguous run of the loop's blocks around its header (a rotated loop's latch
    # sits just before the header), up to the last back-edge; out-of-line blocks (the cosh_glibc
    # fallback) lie beyond it
    h = next(i for i, b in enumerate(blocks) if b[0][4:] == best[0])
    lo = h
    while lo > 0 and inloop(blocks[lo - 1], best):
        lo -= 1
    hi = h
    while hi + 1 < len(blocks) and inloop(blocks[hi + 1], best):
        hi += 1
    heads = "|".join(re.escape(b[0]) for b in blocks[(h if a.first_backedge else lo):h + 1])   # the latch run and the header
    backs = [i for i in range(h, hi + 1) if any(re.search(r"s_(cbranch_\w+|branch)\s+(" + heads + r")\b", x) for x in blocks[i][3])]
    # a bottom-tested loop (its back-edge a conditional branch to the header) ends at its FIRST back-edge;
    # blocks after it that also branch back are out-of-line paths (the cosh_glibc fallback)
    first_cond = [i for i in backs if any(re.search(r"s_cbranch_\w+\s+(" + heads + r")\b", x) for x in blocks[i][3])]
    last = min(first_cond) if (a.first_backedge and first_cond) else max(backs)
    if a.first_backedge:
        lo = h
    seg = [x for b in blocks[lo:last + 1] for x in [b[0] + ":"] + b[3]]
    seg = [x for x in seg if re.match(r"^\s+[a-z]", x) and not x.strip().startswith(";")]
    counts = {}
    for x in seg:
        c = classify(x.strip())
        counts[c] = counts.get(c, 0) + 1
    res = {}
    for key in ("VGPRs", "TotalSGPRs", "ScratchSize", "Occupancy", "LDS Size"):
        m = re.search(re.escape(a.kernel) + r".*?" + re.escape(key) + r"[^:]*: (\d+)", remarks, re.S)
        res[key] = m.group(1) if m else "?"
    print("kernel", a.kernel, "loop header BB%s depth %d" % best, "resources", res)
    print("instructions:", len(seg), counts, "VALU total", counts.get("valu_f64", 0) + counts.get("valu_other", 0))
    if a.dump:
        print("\n".join(seg))


if __name__ == "__main__":
    main()
