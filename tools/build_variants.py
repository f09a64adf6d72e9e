"""Occupancy variants of libcpr_hip for A/B runs (tools/occupancy_ab.sh): the three
event-engine translation units rebuilt with -DCPR_EV_WAVES=<w> (kernels.h), linked with the
default build's other objects into build/var/ev<w>.so; with --ew, -DCPR_EW_WAVES=<w> (the
Ethereum window lane's kernel) into build/var/ew<w>.so; with --roll, -DCPR_ROLL_WAVES=<w>
(k_bk_rollout's wave budget) into build/var/rw<w>.so. Generic A/B variants: --def TAG
TU[,TU] NAME=VAL[,NAME=VAL] rebuilds the named translation units with those macros into
build/var/TAG.so (e.g. --def nolazy kernels.hip CPR_LAZY_CLOCK=0). Every variant a GPU
session loads is built by this script, so its recipe is committed. Run
__graft_entry__.build() first.

Usage: python tools/build_variants.py 2 4;  python tools/build_variants.py --ew 3 4
       python tools/build_variants.py --def nolazy kernels.hip CPR_LAZY_CLOCK=0
"""
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as G  # noqa: E402

# capi.hip is rebuilt in every variant too: it sizes each lane's region with the same
# header functions (bk_lane_bytes, ...) the kernels lay it out with, so a variant that
# changes a lane header must not link the default build's capi.hip.o (round 4's r04o
# illegal memory access: kernels_bk.hip rebuilt alone with a larger vote-record layout)
EV = ["kernels_eth.hip", "kernels_bk.hip", "kernels_ts.hip", "capi.hip"]


def main():
    objdir = ROOT / "build" / "hip"
    out = ROOT / "build" / "var"
    out.mkdir(parents=True, exist_ok=True)
    flags = [f for f in G.HIPCC_FLAGS if f != "-shared"]
    args = sys.argv[1:]
    if args and args[0] == "--def":
        return build_def(objdir, out, flags, args[1], args[2].split(","), args[3].split(","))
    macro, tag = "CPR_EV_WAVES", "ev"
    if args and args[0] == "--ew":
        macro, tag, args = "CPR_EW_WAVES", "ew", args[1:]
    if args and args[0] == "--roll":
        macro, tag, args = "CPR_ROLL_WAVES", "rw", args[1:]
    for w in args:
        vdir = out / f"{tag}{w}"
        vdir.mkdir(exist_ok=True)
        procs = []
        for s in EV:
            cmd = [G._hipcc(), *flags, f"-D{macro}={w}", f"-I{ROOT / 'include'}", "-c",
                   str(G.CSRC / s), "-o", str(vdir / (s + ".o"))]
            procs.append(subprocess.Popen(cmd))
        for p in procs:
            assert p.wait() == 0
        objs = [str((vdir if s in EV else objdir) / (s + ".o"))
                for s in ["kernels.hip", *EV, "kernels_fc16.hip"]]
        subprocess.run([G._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o",
                        str(out / f"{tag}{w}.so")], check=True)
        print("built", out / f"{tag}{w}.so")


ALL = ["kernels.hip", *EV, "kernels_fc16.hip"]


def build_def(objdir, out, flags, tag, tus, defs):
    vdir = out / tag
    vdir.mkdir(exist_ok=True)
    for tu in tus:
        assert tu in ALL, tu
    if "capi.hip" not in tus:
        tus = [*tus, "capi.hip"]  # host sizing from the same headers (see EV)
    procs = [subprocess.Popen([G._hipcc(), *flags, *[f"-D{d}" for d in defs],
                               f"-I{ROOT / 'include'}", "-c", str(G.CSRC / tu), "-o",
                               str(vdir / (tu + ".o"))]) for tu in tus]
    for p in procs:
        assert p.wait() == 0
    objs = [str((vdir if s in tus else objdir) / (s + ".o")) for s in ALL]
    subprocess.run([G._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o",
                    str(out / f"{tag}.so")], check=True)
    print("built", out / f"{tag}.so", "with", " ".join(defs), "in", " ".join(tus))


if __name__ == "__main__":
    main()
