"""LDS bank-conflict audit of the fused PGD tile kernels' access patterns (MI355X_MICROARCH.md §LDS model, via
scripts/ldsbank.py) for a tile geometry (TY x TX outputs, NT threads, blur radius R, fp32).  Prints, per access
site, the worst LDS-array cycles per wave-instruction over all waves and steps against the conflict-free count.
usage: python scripts/ldsbank_tiles.py [TY TX NT R]"""
import sys

sys.path.insert(0, "scripts")
from ldsbank import cost_read_b128  # noqa: E402

G64 = [list(range(0, 32)), list(range(32, 64))]


def cost_read_b64(addrs):
    tot = 0
    for g in G64:
        load = {}
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            for d in range(2):
                load.setdefault((a + d) % 64, set()).add(a + d)
        tot += max([len(v) for v in load.values()] + [1])
    return tot


def cost_write(addrs, width):
    """ds_write_b64 (4 x 16 contiguous lanes) / ds_write_b128 (8 x 8): LDS-array cycles, bank = dword mod 32"""
    glen = 16 if width == 2 else 8
    tot = 0
    for h in range(0, 64, glen):
        load = {}
        for l in range(h, h + glen):
            a = addrs[l]
            if a is None:
                continue
            for d in range(width):
                load.setdefault((a + d) % 32, set()).add(a + d)
        tot += max([len(v) for v in load.values()] + [1])
    return tot


def pad_to(w, m, res, V=4):
    p = w
    while p % m != res:
        p += V
    return p


class Geo:
    def __init__(self, TY, TX, NT, R, pass_b_item=None, stage=None):
        self.TY, self.TX, self.NT, self.R = TY, TX, NT, R
        V = 4
        self.CA = -(-2 * R // V) * V
        self.AR, self.AC = TY + 4 * R, TX + 2 * self.CA
        self.NGA, self.NA, self.NB, self.NCB = self.AC // V, TY // V, self.AC // V, TX // 2
        self.AP = pad_to(self.AC, 32, 28)
        self.PTP = TY + 8
        self.N0, self.NPA, self.NPB = self.AR * self.NGA, self.NA * self.NB, self.NA * self.NCB
        self.pass_b_item = pass_b_item or (lambda it: (it % self.NA, it // self.NA))
        self.stage = stage


def waves(n_items, NT):
    """per wave: list of 64 item indices (None beyond n_items), for items it = tid + k NT"""
    out = []
    for k in range(-(-n_items // NT)):
        for w in range(NT // 64):
            out.append([(t if t < n_items else None) for t in (k * NT + w * 64 + l for l in range(64))])
    return out


def audit(g):
    V, R = 4, g.R
    res = {}

    def rec(name, cost, ideal):
        c, i = res.get(name, (0, ideal))
        res[name] = (max(c, cost), ideal)

    for wv in waves(g.N0, g.NT):  # phase 0: yk window -> A (ds_write_b128)
        addrs = [None if it is None else (it // g.NGA) * g.AP + V * (it % g.NGA) for it in wv]
        rec("phase0 A store (write_b128)", cost_write(addrs, 4), 8)
    for wv in waves(g.NPA, g.NT):  # pass A: sweep reads of A, PT column stores
        for j in range(V + 4 * R):
            addrs = [None if it is None else (V * (it % g.NA) + j) * g.AP + V * (it // g.NA) for it in wv]
            rec("passA A reads (read_b128)", cost_read_b128(addrs), 4)
        for v in range(V):
            addrs = [None if it is None else (V * (it // g.NA) + v) * g.PTP + V * (it % g.NA) for it in wv]
            rec("passA PT stores (write_b128)", cost_write(addrs, 4), 8)
    for wv in waves(g.NPB, g.NT):  # pass B: PT sweep reads, TV window reads of A (ds_read_b64)
        ab = [None if it is None else g.pass_b_item(it) for it in wv]
        for j in range(2 + 4 * R):
            addrs = [None if x is None else (g.CA - 2 * R + 2 * x[1] + j) * g.PTP + V * x[0] for x in ab]
            rec("passB PT reads (read_b128)", cost_read_b128(addrs), 4)
        for r in range(V + 2):
            for off in (-2, 0, 2):
                addrs = [None if x is None else (V * x[0] - 1 + r + 2 * R) * g.AP + g.CA + 2 * x[1] + off for x in ab]
                rec("passB TV A reads (read_b64)", cost_read_b64(addrs), 2)
        if g.stage is not None:
            for u in range(V):
                addrs = [None if x is None else g.stage.idx(V * x[0] + u, 2 * x[1]) for x in ab]
                rec("O stores (write_b64)", cost_write(addrs, 2), 4)
    if g.stage is not None:
        st = g.stage
        for w in range(g.NT // 64):
            lanes = [st.lane(w * 64 + l) for l in range(64)]
            for s in range(g.TY // st.RPS):
                addrs = [st.idx(r0 + s * st.RPS, V * cq) for r0, cq in lanes]
                rec("epilogue O reads (read_b128)", cost_read_b128(addrs), 4)
                addrs = [(r0 + s * st.RPS + 2 * R) * g.AP + g.CA + V * cq for r0, cq in lanes]
                rec("epilogue A reads (read_b128)", cost_read_b128(addrs), 4)
    return res


class Stage64:
    """the current TX = 64 staging layout (tile2d.hpp Stage<float>)"""
    RPS = 256 // 16

    def __init__(self, NT=256):
        self.RPS = NT // 16

    @staticmethod
    def idx(r, c):
        return r * 64 + 4 * (((c >> 2) ^ (2 * (r >> 2))) & 15) + (c & 3)

    @staticmethod
    def lane(tid):
        ln, w = tid & 63, tid >> 6
        h, l = ln >> 5, ln & 31
        if l < 4: g, pos = 0, l
        elif l < 12: g, pos = 1, l - 4
        elif l < 16: g, pos = 0, l - 8
        elif l < 20: g, pos = 1, l - 8
        elif l < 28: g, pos = 0, l - 12
        else: g, pos = 1, l - 16
        return 4 * w + 2 * h + g, pos


def pbi_current(it):  # tile2d.hpp pass_b_item for fp32, NA == 8
    return (it & 3) + 4 * ((it >> 5) & 1), ((it >> 2) & 7) + 8 * (it >> 6)


def report(g, label):
    print(f"== {label}: TY={g.TY} TX={g.TX} NT={g.NT} R={g.R}  AP={g.AP} PTP={g.PTP}  "
          f"items A={g.NPA} B={g.NPB}  LDS A+PT={(g.AR * g.AP + g.AC * g.PTP) * 4} B")
    for k, (c, i) in audit(g).items():
        print(f"   {k:34s} worst {c:3d} cycles (conflict-free {i}){'' if c <= i else '  <-- conflicts'}")


if __name__ == "__main__":
    if len(sys.argv) > 1:
        TY, TX, NT, R = (int(v) for v in sys.argv[1:5])
        report(Geo(TY, TX, NT, R), "generic maps")
    else:
        report(Geo(32, 64, 256, 6, pbi_current, Stage64()), "current tile kernel")


# ----------------------------------------------------------------------------- 64 x 128 tile, 1024 threads
_BQ = {0: 0, 3: 1, 5: 2, 6: 3, 1: 0, 2: 1, 4: 2, 7: 3}
_GQ = {0: 0, 3: 0, 5: 0, 6: 0, 1: 1, 2: 1, 4: 1, 7: 1}


def pa_big(it):
    """pass A item -> (row group a, column group b): per wave 16 row groups x 4 column groups; inside each
    ds_read_b128 lane group 4 consecutive row groups x 4 column groups distinct mod 4"""
    w, l = it >> 6, it & 63
    h, q, lo = l >> 5, (l >> 2) & 7, l & 3
    return lo + 4 * (2 * h + _GQ[q]), _BQ[q] + 4 * w


def pb_big(it):
    """pass B item: the 32 x 64 tile kernel's map inside each quadrant (it >> 8)"""
    qd, i = it >> 8, it & 255
    a, cb = pbi_current(i)
    return a + 8 * (qd >> 1), cb + 32 * (qd & 1)


class StageBig:
    """O = four 32 x 64 quadrants in the tile kernel's layout; epilogue lanes: the tile kernel's map per quadrant"""
    RPS = 16

    @staticmethod
    def idx(r, c):
        qd = (r // 32) * 2 + (c // 64)
        return qd * 2048 + Stage64.idx(r % 32, c % 64)

    @staticmethod
    def lane(tid):
        qd, t = tid >> 8, tid & 255
        r0, cq = Stage64.lane(t)
        return r0 + 32 * (qd >> 1), cq + 16 * (qd & 1)


def audit_big(R=6):
    g = Geo(64, 128, 1024, R, pb_big, None)
    V = 4
    res = {}

    def rec(name, cost, ideal):
        c, _ = res.get(name, (0, ideal))
        res[name] = (max(c, cost), ideal)

    for wv in waves(g.NA * 4 * 10, g.NT):  # pass A with pa_big (items beyond NB column groups idle)
        ab = [None if it is None else pa_big(it) for it in wv]
        ab = [None if (x is None or x[1] >= g.NB) else x for x in ab]
        for j in range(V + 4 * R):
            rec("passA A reads (read_b128)", cost_read_b128([None if x is None else (V * x[0] + j) * g.AP + V * x[1] for x in ab]), 4)
        for v in range(V):
            rec("passA PT stores (write_b128)", cost_write([None if x is None else (V * x[1] + v) * g.PTP + V * x[0] for x in ab], 4), 8)
    for wv in waves(g.NPB, g.NT):
        ab = [None if it is None else pb_big(it) for it in wv]
        for j in range(2 + 4 * R):
            rec("passB PT reads (read_b128)", cost_read_b128([None if x is None else (g.CA - 2 * R + 2 * x[1] + j) * g.PTP + V * x[0] for x in ab]), 4)
        for r in range(V + 2):
            for off in (-2, 0, 2):
                rec("passB TV A reads (read_b64)", cost_read_b64([None if x is None else (V * x[0] - 1 + r + 2 * R) * g.AP + g.CA + 2 * x[1] + off for x in ab]), 2)
        for u in range(V):
            rec("O stores (write_b64)", cost_write([None if x is None else StageBig.idx(V * x[0] + u, 2 * x[1]) for x in ab], 2), 4)
    for w in range(16):
        lanes = [StageBig.lane(w * 64 + l) for l in range(64)]
        for s in range(2):
            rec("epilogue O reads (read_b128)", cost_read_b128([StageBig.idx(r0 + 16 * s, V * cq) for r0, cq in lanes]), 4)
            rec("epilogue A reads (read_b128)", cost_read_b128([(r0 + 16 * s + 2 * R) * g.AP + g.CA + V * cq for r0, cq in lanes]), 4)
    # coverage checks
    itemsA = sorted(pa_big(it) for it in range(1024) if pa_big(it)[1] < g.NB)
    assert itemsA == sorted((a, b) for a in range(g.NA) for b in range(g.NB)), "pass A map"
    itemsB = sorted(pb_big(it) for it in range(1024))
    assert itemsB == sorted((a, c) for a in range(g.NA) for c in range(g.NCB)), "pass B map"
    pix = sorted((r0 + 16 * s, cq) for t in range(1024) for s in range(2) for r0, cq in [StageBig.lane(t)])
    assert pix == sorted((r, c) for r in range(64) for c in range(32)), "epilogue map"
    print(f"== big tile 64 x 128, 1024 threads, R={R}: AP={g.AP} PTP={g.PTP} LDS A={g.AR * g.AP * 4} PT={g.AC * g.PTP * 4}")
    for k, (c, i) in res.items():
        print(f"   {k:34s} worst {c:3d} cycles (conflict-free {i}){'' if c <= i else '  <-- conflicts'}")
