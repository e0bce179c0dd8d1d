"""Cost model of b3_leaf_kernel's wave schedule on the zipf10k chunk-length mix.
Unit: one wave-wide compress (= one 64-lane issue of the compress body)."""
import sys, numpy as np
sys.path.insert(0, "/root/repo")
import bench
rng = np.random.default_rng(1)
sizes, _, _ = bench.workload("zipf10k", 1)
CAP, P = 2 << 20, 2.0 ** -20
lens = []
for s in sizes.astype(np.int64):
    pos = 0
    while pos < s:
        seg = min(CAP, s - pos)          # one read of the production loop
        q = 0
        while q < seg:
            g = int(rng.geometric(P))
            if q + g >= seg:
                lens.append(seg - q); break
            lens.append(g); q += g
        pos += seg
lens = np.array(lens, np.int64)
print("chunks", lens.size, "bytes", lens.sum(), "mean KiB", lens.mean() / 1024)
LPL = int(sys.argv[1]) if len(sys.argv) > 1 else 4
def tasks(n): return max(1, -(-max(1, -(-n // 1024)) // LPL))
def task_blocks(n, k):      # blocks of task k of a chunk of n bytes
    b = max(0, min(1024 * LPL, n - k * 1024 * LPL))
    return max(1, -(-b // 64))
ideal = (np.maximum(1, -(-lens // 64))).sum() / 64.0     # data blocks / 64 lanes
def wave_cost(lane_blocks, levels):
    mb = max(lane_blocks)
    nl = -(-mb // 16)
    fold = {1: 0, 2: 1, 3: 2, 4: 3}.get(nl, nl - 1) if LPL == 4 else max(0, nl - 1)
    return mb + fold + levels
def ceil_log2(t): return 0 if t <= 1 else int(t - 1).bit_length()
def run(tail_pack):
    cost = 0.0
    classes = {c: [] for c in range(7)}
    for n in lens.tolist():
        t = tasks(n)
        if t <= 64:
            classes[ceil_log2(t)].append((n, 0, t))
            continue
        full, tail = divmod(t, 64)
        for g in range(full):
            cost += wave_cost([task_blocks(n, g * 64 + l) for l in range(64)], 6)
        if tail:
            if tail_pack: classes[ceil_log2(tail)].append((n, full * 64, tail))
            else: cost += wave_cost([task_blocks(n, full * 64 + l) for l in range(tail)], 6)
    for c, lst in classes.items():
        per = 64 >> c
        for i in range(0, len(lst), per):
            lb = []
            for (n, k0, t) in lst[i:i + per]:
                lb += [task_blocks(n, k0 + l) for l in range(t)]
            cost += wave_cost(lb, c)
    return cost
base = run(False); tp = run(True)
print(f"LPL {LPL}: ideal {ideal:.0f}  current {base:.0f} ({base/ideal:.3f}x)  tail-packed {tp:.0f} ({tp/ideal:.3f}x)")

def run2(pack, defer, sort_desc=False):
    """pack: 'class' | 'firstfit'; defer: merges of more than one task done by a
    level-synchronous tree pass (cost = parents/64 per level) instead of in-wave."""
    data = fold = merge = 0.0
    units = []          # (n, k0, t, wave_root)
    for n in lens.tolist():
        t = tasks(n)
        if t <= 64: units.append((n, 0, t)); continue
        full, tail = divmod(t, 64)
        for g in range(full): units.append((n, g * 64, 64))
        if tail: units.append((n, full * 64, tail))
    waves = []
    if pack == "class":
        cl = {c: [] for c in range(7)}
        for u in units: cl[ceil_log2(u[2])].append(u)
        for c, lst in cl.items():
            per = 64 >> c
            for i in range(0, len(lst), per): waves.append((lst[i:i + per], c))
    else:
        us = sorted(units, key=lambda u: -u[2]) if sort_desc else units
        cur, used = [], 0
        for u in us:
            if used + u[2] > 64:
                waves.append((cur, None)); cur, used = [], 0
            cur.append(u); used += u[2]
        if cur: waves.append((cur, None))
    for lst, c in waves:
        lb = []
        for (n, k0, t) in lst: lb += [task_blocks(n, k0 + l) for l in range(t)]
        mb = max(lb); nl = -(-mb // 16)
        data += mb; fold += max(0, nl - 1)
        lv = c if c is not None else ceil_log2(max(u[2] for u in lst))
        if not defer: merge += lv
    if defer:   # level-synchronous: every level packs all pending parents of all chunks
        cnt = [tasks(n) for n in lens.tolist()]
        while True:
            par = sum(x // 2 for x in cnt)
            if par == 0: break
            merge += -(-par // 64)
            cnt = [-(-x // 2) for x in cnt]
    tot = data + fold + merge
    print(f"  {pack:8s} defer={defer} sort={sort_desc}: data {data/ideal:.3f} fold {fold/ideal:.3f} merge {merge/ideal:.3f} total {tot/ideal:.3f}x")
for pack in ("class", "firstfit"):
    for defer in (False, True):
        run2(pack, defer)
run2("firstfit", False, True); run2("firstfit", True, True)

def run3():
    """class packing incl. tails (in-wave merges for packed units); group items
    write 64 task CVs; one tree wave per big chunk merges level by level."""
    data = fold = merge = tree = 0.0
    cl = {c: [] for c in range(7)}
    for n in lens.tolist():
        t = tasks(n)
        if t <= 64: cl[ceil_log2(t)].append((n, 0, t)); continue
        full, tail = divmod(t, 64)
        for g in range(full):
            lb = [task_blocks(n, g * 64 + l) for l in range(64)]
            mb = max(lb); data += mb; fold += max(0, -(-mb // 16) - 1)
        if tail: cl[ceil_log2(tail)].append((n, full * 64, tail))
        x = full * 64 + (1 if tail else 0)     # tree nodes: task CVs + tail subtree
        # level pairing over tasks; the tail CV is a level-6 node -- model as plain pairing
        nodes = full * 64 + (64 if tail else 0)
        while nodes > 1:
            par = nodes // 2
            tree += -(-par // 64)
            nodes = -(-nodes // 2)
    for c, lst in cl.items():
        per = 64 >> c
        for i in range(0, len(lst), per):
            lb = []
            for (n, k0, t) in lst[i:i + per]: lb += [task_blocks(n, k0 + l) for l in range(t)]
            mb = max(lb); data += mb; fold += max(0, -(-mb // 16) - 1); merge += c
    tot = data + fold + merge + tree
    print(f"  run3: data {data/ideal:.3f} fold {fold/ideal:.3f} merge {merge/ideal:.3f} tree {tree/ideal:.3f} total {tot/ideal:.3f}x")
run3()
