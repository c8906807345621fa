"""Build the MI355X extension in-tree: ppls_amd/_build/libaquad.so (+ the `aquad` CLI).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build container as well as on
the GPU box. Flags that matter for parity:
  -ffp-contract=off  the reference was compiled for baseline x86-64 (no FMA contraction); every
                     fusion the device libm needs is an explicit __fma_rn() (aq_libm.h).
  no -ffast-math     IEEE-correct f64 division (v_div_scale / v_div_fmas / v_div_fixup).
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libaquad.so")
CLI = os.path.join(OUT, "aquad")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ARCH = os.environ.get("PPLS_AMD_ARCH", "gfx950")

# -amdgpu-atomic-optimizer-strategy=None: every device atomic here is already issued by one lane (the
# kernels aggregate by hand); LLVM's optimizer wraps each in a ballot / mbcnt / readfirstlane sequence
# whose broadcast of the returned value waits for the atomic at once -- it had made k_stream's job
# claim (meant to stay in flight across a job) a full round trip. r02 A/B: bench -1.5 %, lone
# integral 26.5 -> 25.7 us (profiles/r02_ab/sload_atomic_opt.txt).
HIP_FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
             "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
             "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include"), "-I", CSRC]

SOURCES = [os.path.join(CSRC, "aquad.hip")]
# AQ_F_USER plug-in header (the reference's F(arg) macro, aquadPartA.c:46): the default Gaussian,
# or any header named by PPLS_AMD_USER_F (see csrc/plugins/aq_user_gauss.h for the interface)
USER_F = os.path.abspath(os.environ.get("PPLS_AMD_USER_F") or os.path.join(CSRC, "plugins", "aq_user_gauss.h"))
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("aq_libm.h", "aq_exp_table.h", "aq_sincos_table.h", "aq_device.h", "aq_stream.h",
                                                  "aq_xsum.h", "aq_abi.inc")] + \
    [os.path.join(ROOT, "include", "aquad.h"), USER_F]
LIBS = ["-pthread", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_variant(name, defines, verbose=False):
    """An A/B variant of the library with extra -D flags: _build/libaquad_<name>.so (tools/ab.sh)."""
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, f"libaquad_{name}.so")
    cmd = [HIPCC] + HIP_FLAGS + [f'-DAQ_USER_F_HEADER="{USER_F}"'] + list(defines) + ["-o", out] + SOURCES + LIBS
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return out


def build(force=False, verbose=False):
    os.makedirs(OUT, exist_ok=True)
    tab = os.path.join(CSRC, "aq_exp_table.h")
    if not os.path.exists(tab):
        subprocess.check_call([sys.executable, os.path.join(CSRC, "gen_exp_table.py")])
    if not os.path.exists(os.path.join(CSRC, "aq_sincos_table.h")):
        subprocess.check_call([sys.executable, os.path.join(CSRC, "gen_sincos_table.py")])
    if force or _stale(LIB, DEPS):
        cmd = [HIPCC] + HIP_FLAGS + [f'-DAQ_USER_F_HEADER="{USER_F}"', "-o", LIB] + SOURCES + LIBS
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    cli_src = os.path.join(CSRC, "aquad_cli.c")
    if os.path.exists(cli_src) and (force or _stale(CLI, [cli_src, LIB])):
        cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-I", os.path.join(ROOT, "include"), "-o", CLI, cli_src,
               "-L", OUT, "-laquad", "-Wl,-rpath,$ORIGIN", "-lm"]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    if "--variant" in sys.argv:   # python ppls_amd/build.py --variant NAME [-DX=1 ...]
        i = sys.argv.index("--variant")
        # -D... defines, and --mllvm=<option> for LLVM options (scheduler experiments)
        extra = []
        for a in sys.argv[i + 2:]:
            if a.startswith("-D"):
                extra.append(a)
            elif a.startswith("--mllvm="):
                extra += ["-mllvm", a[len("--mllvm="):]]
            elif a.startswith("-f"):   # code-generation flags (e.g. -falign-loops=64)
                extra.append(a)
        print("built", build_variant(sys.argv[i + 1], extra))
    else:
        build(force="--force" in sys.argv, verbose=True)
        print("built", LIB)
