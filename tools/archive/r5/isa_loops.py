"""Instruction mix of a kernel's loops in the gfx950 ISA (development aid for
the VALU-bound path loops): compiles csrc/<file> to assembly (device only)
with the LM shape list cut down to ONE shape (a patched copy in a temp dir,
so hedge_lm.hip compiles in ~1 min instead of 5), finds every loop
(back-edge) of the kernel whose mangled name contains KEY, and prints its
instruction count by class and the most frequent opcodes.

usage: python tools/archive/r5/isa_loops.py FILE KEY [--shape 1,8,2,HEAD_FREE] [--keep DIR]
  e.g. python tools/archive/r5/isa_loops.py hedge_lm.hip 'k_lm_passINS_14NarrowPairBodyILi1ELi8ELi2ELi0ELb0E'"""
import argparse
import collections
import re
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]


def compile_asm(src_name: str, shape: str, out_dir: Path) -> Path:
    src_dir = out_dir / "csrc"
    shutil.copytree(ROOT / "csrc", src_dir)
    f = src_dir / src_name
    if src_name == "hedge_lm.hip" and shape:
        s = f.read_text()
        i = s.index("#define RPH_LM_SHAPES(X)")
        j = s.index("\n\n", i)
        s = s[:i] + f"#define RPH_LM_SHAPES(X) X({shape})" + s[j:]
        f.write_text(s)
    out = out_dir / (src_name + ".s")
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{src_dir}", "--cuda-device-only", "-S"]
    if src_name == "hedge_lm.hip":
        flags += ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-o", str(out), str(f)], check=True)
    return out


def loops(asm: Path, key: str):
    lines = asm.read_text().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and key in l]
    for st in starts:
        name = lines[st].split(":")[0]
        end = st + next(i for i, l in enumerate(lines[st:]) if l.strip().startswith(".Lfunc_end"))
        body = lines[st:end]
        labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}

        def is_ins(x):
            s = x.strip()
            return s and not s.startswith((";", ".")) and not s.endswith(":")

        print(name)
        for i, l in enumerate(body):
            m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
            if not m or m.group(1) not in labels or labels[m.group(1)] >= i:
                continue
            ins = [x.strip().split()[0] for x in body[labels[m.group(1)]:i + 1] if is_ins(x)]
            if len(ins) < 40:
                continue
            c = collections.Counter(ins)
            cls = {k: sum(v for o, v in c.items() if o.startswith(p)) for k, p in
                   (("valu", "v_"), ("pk", "v_pk"), ("mov", "v_mov"), ("agpr", "v_accvgpr"), ("ds", "ds_"),
                    ("vmem", ("global_", "buffer_")), ("salu", "s_"))}
            print(f"  loop {m.group(1)}: {len(ins)} instrs", cls, "nop", c["s_nop"])
            print("    ", c.most_common(12))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("key")
    ap.add_argument("--shape", default="1, 8, 2, HEAD_FREE")
    ap.add_argument("--keep", default=None)
    a = ap.parse_args()
    d = Path(a.keep) if a.keep else Path(tempfile.mkdtemp())
    d.mkdir(parents=True, exist_ok=True)
    if (d / "csrc").exists():
        shutil.rmtree(d / "csrc")
    asm = compile_asm(a.file, a.shape.replace(",", ", ").replace("  ", " "), d)
    loops(asm, a.key)
    if not a.keep:
        shutil.rmtree(d)


if __name__ == "__main__":
    sys.exit(main())
