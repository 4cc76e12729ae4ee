"""PMC passes (tools/pmc_run.sh) -> HBM bytes per launch / per step, as
profiles/pmc_traffic.json entries {"bytes", "src", "file"}: "src" is the hash
of the kernel sources measured (bench.py kernel_src_hash), so bench.py reports
them only while those sources are unchanged.  HBM bytes = 2·FETCH_SIZE +
WRITE_SIZE (KB; FETCH_SIZE counts half of a wide streaming read on gfx950,
MI355X_MICROARCH.md HBM section).

    python3 tools/pmc_traffic.py gpurun_out/pmc [--merge profiles/pmc_traffic.json --file profiles/r07/pmc.txt]
"""
import collections
import csv
import glob
import importlib.util
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(HERE, "..", "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def load(d, ctr):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        for r in rows:
            if r.get("Counter_Name") == ctr:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024)
    return acc


def pick(acc, pats):
    """The kernel whose name holds any of ``pats`` (mangled or demangled)."""
    pats = (pats,) if isinstance(pats, str) else pats
    ks = [k for k in acc if any(p in k for p in pats)]
    return ks[0] if ks else None


def main():
    d = sys.argv[1]
    b = _bench()
    out, lines = {}, []
    # the head's passes: mean over the launches
    F, W = load(os.path.join(d, "head_FETCH_SIZE"), "FETCH_SIZE"), load(os.path.join(d, "head_WRITE_SIZE"), "WRITE_SIZE")
    for key, pat in (("head_fwd:f32x6d3:zs", ("k_flash_fwdILi128ELi6ELi3ELi0ELb1EE", "k_flash_fwd<128, 6, 3, 0, true>")),
                     ("head_dw_adam:f32x6d3:zs", ("k_flash_dwILi128ELi6ELb1EE", "k_flash_dw<128, 6, true>"))):
        kf, kw = pick(F, pat), pick(W, pat)
        if kf is None or kw is None:
            lines.append(f"{key}: kernel {pat} not found")
            continue
        f, w = sum(F[kf]) / len(F[kf]), sum(W[kw]) / len(W[kw])
        out[key] = {"bytes": int(2 * f + w), "src": b.kernel_src_hash("head")}
        lines.append(f"{key}: fetch {f / 1e9:.3f} GB x2 + write {w / 1e9:.3f} GB = {(2 * f + w) / 1e9:.3f} GB per "
                     f"launch ({len(F[kf])} launches, {kf[:60]})")
    # the north-star kernels: the last step's launches (one gather at C2, the two directions' at C3)
    for cfg, ng in (("c2", 1), ("c3", 2)):
        F = load(os.path.join(d, f"ns_{cfg}_FETCH_SIZE"), "FETCH_SIZE")
        W = load(os.path.join(d, f"ns_{cfg}_WRITE_SIZE"), "WRITE_SIZE")
        tot, parts = 0.0, []
        for pat, n in (("k_gather_e", ng), ("k_sampled_logits", 1)):
            kf, kw = pick(F, pat), pick(W, pat)
            if kf is None or kw is None:
                parts = None
                break
            f, w = sum(F[kf][-n:]), sum(W[kw][-n:])
            tot += 2 * f + w
            parts.append(f"{pat} x{n}: fetch {f / 1e6:.1f} MB x2 + write {w / 1e6:.1f} MB")
        key = f"{cfg}:gather+sampled_fwd"
        if parts is None:
            lines.append(f"{key}: kernels not found")
            continue
        out[key] = {"bytes": int(tot), "src": b.kernel_src_hash("gather+sampled_fwd")}
        lines.append(f"{key}: {'; '.join(parts)} = {tot / 1e6:.1f} MB per step")
    print("\n".join(lines))
    print(json.dumps(out))
    if "--merge" in sys.argv:
        tab_path = sys.argv[sys.argv.index("--merge") + 1]
        ref = sys.argv[sys.argv.index("--file") + 1] if "--file" in sys.argv else None
        tab = json.load(open(tab_path))
        for k, v in out.items():
            tab[k] = dict(v, file=ref)
        json.dump(tab, open(tab_path, "w"), indent=1)


if __name__ == "__main__":
    main()
