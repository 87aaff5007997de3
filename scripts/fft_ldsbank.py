"""LDS bank model (MI355X_MICROARCH.md §LDS table) for the in-place FFT kernel's stage reads / writes and its
line load / store orders: conflict degree (max lanes on one bank) per access pattern, for the fp32 plans of
factor_lds and candidate swizzles.  usage: python scripts/fft_ldsbank.py"""
import collections


def padi(i):
    return i ^ ((i >> 3) & 15)


def pitch(n, L):
    return n + 16 // min(L, 16)


def plan(n, esize=8):
    out, r0 = [], 16 if esize == 8 else 8
    for r in (r0, 8, 4, 2):
        while n % r == 0:
            out.append(r)
            n //= r
    return out


def ways(elems, groups, nslots):
    worst = 1
    for g in groups:
        load = collections.defaultdict(set)
        for lane in g:
            if elems[lane] is not None:
                load[elems[lane] % nslots].add(elems[lane])
        worst = max([worst] + [len(v) for v in load.values()])
    return worst


RD = [list(range(0, 32)), list(range(32, 64))]          # ds_read_b64: 2 x 32, 8-B slot mod 32
WR = [list(range(h, h + 16)) for h in range(0, 64, 16)]  # ds_write_b64: 4 x 16, 8-B slot mod 16


def stage_ways(n, L, R, ns, sw, TH=512):
    P = pitch(n, L)
    nr = n // R
    total = L * nr
    worst_r, worst_w = 1, 1
    for wave in range(TH // 64):
        for b in range((16 + R - 1) // R):
            for r in range(R):
                rd, wr = [], []
                for lane in range(64):
                    t = wave * 64 + lane + b * TH
                    if t >= total:
                        rd.append(None)
                        wr.append(None)
                        continue
                    l, j = t // nr, t % nr
                    k = j % ns
                    idn = (j - k) * R + k
                    rd.append(l * P + sw(j + r * nr))
                    wr.append(l * P + sw(idn + r * ns))
                worst_r = max(worst_r, ways(rd, RD, 32))
                worst_w = max(worst_w, ways(wr, WR, 16))
    return worst_r, worst_w


def main():
    for name, sw in (("padi", padi),):
        for n in (64, 256, 1024, 2048, 4096, 8192):
            L = max(1, 8192 // n)
            ns = 1
            rows = []
            for R in plan(n):
                rows.append((R, ns) + stage_ways(n, L, R, ns, sw))
                ns *= R
            print(name, n, "L", L, " ".join(f"R{R}@ns{s}:r{a}w{b}" for R, s, a, b in rows))


if __name__ == "__main__":
    main()
