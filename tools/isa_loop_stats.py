"""Static instruction mix of the activation loop of a fused-episode kernel.

Compiles one translation unit to gfx950 assembly (hipcc -S, same flags as the build),
finds the kernel, and counts the instructions of every basic block whose innermost loop
is the activation loop (the depth-2 loop: depth 1 is the grid-stride episode loop),
plus those of loops nested in it, separately. Used to compare layouts of the Nakamoto
lane without a GPU; the PMC-measured SQ_INSTS_VALU per activation is the real figure.

usage: python tools/isa_loop_stats.py [kernels.hip] [kernel-substring] [-D...] [--by-source]

--by-source compiles with -g as well and splits the activation loop's VALU instructions by
the source function their .loc line falls in (inlined callees keep their own lines): the
static cost-centre breakdown of one iteration (Philox, log, policy, apply, resolve, ...).
"""
import collections
import pathlib
import re
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent


def compile_asm(src, defines, debug=False):
    out = pathlib.Path("/tmp") / (pathlib.Path(src).stem + ("_g" if debug else "") + ".s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-ffp-contract=off", f"-I{ROOT / 'include'}", "--cuda-device-only", "-S",
           *(["-g"] if debug else []), *defines, str(src), "-o", str(out)]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return out.read_text().split("\n")


def kernel_meta(lines, name):
    meta = {}
    for i, l in enumerate(lines):
        if l.strip() == f".name:           {name}":
            for l2 in lines[i - 12:i + 12]:
                m = re.match(r"\s+\.(sgpr_count|vgpr_count|sgpr_spill_count|vgpr_spill_count|"
                             r"private_segment_fixed_size):\s+(\d+)", l2)
                if m:
                    meta[m.group(1)] = int(m.group(2))
    return meta


def kernel_lines(lines, sub):
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l)]
    for j, s in enumerate(starts):
        if sub in lines[s]:
            e = starts[j + 1] if j + 1 < len(starts) else len(lines)
            return lines[s:e], lines[s].split(":")[0]
    raise SystemExit(f"kernel {sub!r} not found")


FUNC_RE = re.compile(r"(?:inline|__device__|__global__)[^;{()]*?\b([A-Za-z_]\w*)\s*\(")


def func_table(path):
    """(line, function) of every function head in a source file, ascending"""
    out = []
    try:
        text = pathlib.Path(path).read_text().split("\n")
    except OSError:
        return out
    for i, l in enumerate(text, 1):
        m = FUNC_RE.search(l)
        if m and m.group(1) not in ("if", "for", "while", "return", "sizeof"):
            out.append((i, m.group(1)))
    return out


def by_source(all_lines, lines, loop_labels):
    files = {}
    for l in all_lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(2) + "/" + m.group(3)) if m.group(3) else m.group(2)
    tables = {}
    cur = None
    inloop = False
    cnt = collections.Counter()
    for l in lines:
        m = re.match(r"^(\.L(BB\d+_\d+):|; %bb\.\d+:)(.*)$", l)
        if m:
            lab = m.group(2)
            ann = m.group(3)
            mm = re.search(r"in Loop: Header=(BB\d+_\d+)", ann)
            inloop = (lab in loop_labels) or (mm is not None and mm.group(1) in loop_labels)
            continue
        t = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (m.group(1), int(m.group(2)))
            continue
        if not inloop or not t.startswith("v_") or cur is None or cur[1] == 0:
            continue
        path = files.get(cur[0], "?")
        if path not in tables:
            tables[path] = func_table(path)
        fn = "?"
        for ln, name in tables[path]:
            if ln <= cur[1]:
                fn = name
            else:
                break
        cnt[(pathlib.Path(path).name, fn)] += 1
    total = sum(cnt.values())
    print(f" VALU by source function (loop body, {total} instructions):")
    for (f, fn), c in cnt.most_common(40):
        print(f"   {c:4d} {100.0 * c / max(1, total):5.1f}%  {f}:{fn}")


def main():
    dbg = "--by-source" in sys.argv
    args = [a for a in sys.argv[1:] if not a.startswith("-")]
    defines = [a for a in sys.argv[1:] if a.startswith("-D")]
    src = args[0] if args else str(ROOT / "cpr_amd" / "csrc" / "kernels.hip")
    sub = args[1] if len(args) > 1 else "k_run_episodesILi0ENS_10SeedSourceELi3E"
    all_lines = compile_asm(src, defines, dbg)
    lines, name = kernel_lines(all_lines, sub)
    meta = kernel_meta(all_lines, name)
    # basic blocks: (label, annotation comments, instructions)
    blocks = []
    for l in lines:
        m = re.match(r"^(\.L(BB\d+_\d+):|; %bb\.\d+:)(.*)$", l)
        if m:
            blocks.append([m.group(2), m.group(3), []])
            continue
        t = l.strip()
        if not blocks:
            continue
        if t.startswith(";") and not blocks[-1][2]:
            blocks[-1][1] += " " + t
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        blocks[-1][2].append(t.split()[0])
    depth = {}
    for lab, ann, _ in blocks:
        m = re.search(r"This Loop Header: Depth=(\d+)", ann)
        if m:
            depth[lab] = int(m.group(1))
    hdr2 = [h for h, d in depth.items() if d == 2]
    per = {h: collections.Counter() for h in hdr2}
    nested = collections.Counter()
    for lab, ann, ins in blocks:
        if lab in depth:
            loop = lab
        else:
            m = re.search(r"in Loop: Header=(BB\d+_\d+)", ann)
            loop = m.group(1) if m else None
        if loop in per:
            per[loop].update(ins)
        elif loop is not None and depth.get(loop, 0) > 2:
            nested.update(ins)
    # the activation loop: the depth-2 loop with the most Philox multiplies (several
    # depth-2 loops exist when run_gym has a uniform and a general variant; report the
    # largest, which the bench's configuration runs)
    for h, c in sorted(per.items(), key=lambda x: -sum(v for o, v in x[1].items()
                                                       if o.startswith("v_"))):
        print(f" depth-2 loop {h}: VALU {sum(v for o, v in c.items() if o.startswith('v_'))}")
    # the first depth-2 loop in block order is run_gym's uniform-trip-count loop (the
    # configuration the bench runs: only max_steps ends an episode)
    body = per[hdr2[0]] if hdr2 else collections.Counter()
    v = sum(c for o, c in body.items() if o.startswith("v_"))
    s = sum(c for o, c in body.items() if o.startswith("s_"))
    mov = sum(c for o, c in body.items() if o.startswith("v_mov"))
    lane = sum(c for o, c in body.items() if "lane" in o and o.startswith("v_"))
    f64 = sum(c for o, c in body.items() if o.startswith("v_") and "f64" in o)
    print(f"{name}\n activation-loop body: VALU {v} (v_mov {mov}, readlane/writelane {lane}, "
          f"f64 {f64}), SALU {s}, LDS {sum(c for o, c in body.items() if o.startswith('ds_'))}")
    nv = sum(c for o, c in nested.items() if o.startswith("v_"))
    print(f" registers: {meta}")
    print(f" nested loops inside it: VALU {nv}")
    for o, c in body.most_common(25):
        print(f"   {c:4d} {o}")
    if dbg and hdr2:
        # the loop body: its header block and every block annotated as in that loop
        by_source(all_lines, lines, {hdr2[0]})


if __name__ == "__main__":
    main()
