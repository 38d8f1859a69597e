"""Build a measurement variant of liblsr.so with extra compile flags (same-box A/B comparisons).

    python tools/build_variant.py <name> -DFOO=0 [...]   ->  langsplat_amd/liblsr_<name>.so
    python tools/build_variant.py <name> --rev <git rev>  ->  the sources of that commit

Load it with LSR_LIB=langsplat_amd/liblsr_<name>.so (langsplat_amd/_native.py); the product path
always loads langsplat_amd/liblsr.so.
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from langsplat_amd import build as B  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    csrc = B.CSRC
    if extra[:1] == ["--rev"]:  # the sources (csrc/ + include/) of an earlier commit
        rev, extra = extra[1], extra[2:]
        tmp = tempfile.mkdtemp(prefix="lsr_rev_")
        arc = subprocess.run(["git", "-C", ROOT, "archive", rev, "langsplat_amd/csrc", "include"], check=True,
                             capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", tmp], input=arc, check=True)
        csrc = os.path.join(tmp, "langsplat_amd", "csrc")
    out_dir = os.path.join(ROOT, "build", f"variant_{name}")
    os.makedirs(out_dir, exist_ok=True)
    cc = B.hipcc()
    objs = []
    for src in B.SOURCES:
        obj = os.path.join(out_dir, src.replace(".hip", ".o"))
        subprocess.run([cc] + B.cflags() + B.EXTRA_FLAGS.get(src, []) + extra + ["-c", os.path.join(csrc, src), "-o",
                                                                                 obj], check=True)
        objs.append(obj)
    lib = os.path.join(B.HERE, f"liblsr_{name}.so")
    subprocess.run([cc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
