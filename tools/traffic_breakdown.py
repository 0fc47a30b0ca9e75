"""Per-level HBM traffic of the bench's DenseLayer convs against their algorithmic bytes, from
a committed PMC capture (tools/pmc_bench.sh: FETCH_SIZE and WRITE_SIZE passes over one
`bench.py --steps 1 --warmup 1 --no-residual` run).  The last 213 conv dispatches of the capture
are the sampled encode of bench.roofline_pass (imagenet64, B = 256): level 0's 8 couplings and
prior as 12 per-layer launches each, level 1's 9 blocks as one fused launch each, level 2's 8
couplings as 12 launches each (its prior is the cached top prior).  Algorithmic bytes per layer
as bench.conv_algorithmic_bytes: 4 B x (c + g) per pixel + the 9 x c x g weight pairs.
HBM bytes = 2 x FETCH_SIZE (the gfx950 correction) + WRITE_SIZE, KiB.  Analysis tool (CPU)."""
import csv
import gzip
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
KERNELS = ("conv3_dx3_kernel<3,", "conv3_dx3_block_kernel<3,")


def blocks_in_encode_order():
    from idfcodec import configs, synthetic
    sd = synthetic.build_model(configs.get("imagenet64")).state_dict()
    out = []  # (level, name, [(c, g) per layer])
    for k in sd:
        m = re.match(r"blocks\.(\d)\.(.*)\.layers\.0\.layers\.1\.weight$", k)
        if not m:
            continue
        lvl, name = int(m.group(1)), m.group(2)
        pre = k[: -len("layers.0.layers.1.weight")]
        layers, i = [], 0
        while f"{pre}layers.{i}.layers.1.weight" in sd:
            g, c = sd[f"{pre}layers.{i}.layers.1.weight"].shape[:2]
            layers.append((int(c), int(g)))
            i += 1
        if lvl == 2 and name.startswith("prior"):
            continue  # the cached top prior
        out.append((lvl, name, layers))
    return out


def rows(path):
    with gzip.open(path, "rt", newline="") as f:
        r = sorted(csv.DictReader(f), key=lambda r: int(r["Dispatch_Id"]))
    return [x for x in r if any(k in x["Kernel_Name"] for k in KERNELS)]


def main(d=os.path.join(REPO, "profiles", "r06", "pmc_bench")):
    fetch, write = rows(os.path.join(d, "fetch.csv.gz")), rows(os.path.join(d, "write.csv.gz"))
    B, hw = 256, {0: 32 * 32, 1: 16 * 16, 2: 8 * 8}
    launches = []  # (level, c of the launch's first layer, algorithmic bytes)
    for lvl, name, layers in blocks_in_encode_order():
        P = B * hw[lvl]
        per = [(c, 4 * P * (c + g) + 9 * c * g * 4) for c, g in layers]
        if lvl == 1:  # the fused DenseBlock: one launch
            launches.append((lvl, per[0][0], sum(b for _, b in per)))
        else:
            launches += [(lvl, c, b) for c, b in per]
    n = len(launches)
    fetch, write = fetch[-n:], write[-n:]
    assert len(fetch) == n and len(write) == n, (len(fetch), n)
    tot = {}
    for (lvl, c, algo), f, w in zip(launches, fetch, write):
        hbm = (2 * float(f["Counter_Value"]) + float(w["Counter_Value"])) * 1024
        t = tot.setdefault(lvl, [0, 0.0, 0.0, {}])
        t[0] += 1
        t[1] += algo
        t[2] += hbm
        if lvl == 0:
            t[3].setdefault(c, [0.0, 0.0])
            t[3][c][0] += algo
            t[3][c][1] += hbm
    print(f"{n} launches (source_hash {open(os.path.join(d, 'source_hash.txt')).read()[:16]})")
    A = sum(t[1] for t in tot.values())
    H = sum(t[2] for t in tot.values())
    for lvl, (cnt, algo, hbm, _) in sorted(tot.items()):
        print(f"level {lvl}: {cnt:3d} launches, algorithmic {algo / 1e9:7.2f} GB, HBM {hbm / 1e9:7.2f} GB, "
              f"ratio {hbm / algo:.3f}, excess {100 * (hbm - algo) / (H - A):5.1f}% of the total excess")
    print(f"all: algorithmic {A / 1e9:.2f} GB, HBM {H / 1e9:.2f} GB, ratio {H / A:.3f}, "
          f"per launch {H / n / 1e6:.1f} / {A / n / 1e6:.1f} MB")
    print("level 0 by layer input channels c (8 couplings + prior summed):")
    for c, (algo, hbm) in sorted(tot[0][3].items()):
        print(f"  c = {c:4d}: algorithmic {algo / 1e6:8.1f} MB, HBM {hbm / 1e6:8.1f} MB, ratio {hbm / algo:.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
