"""CPU trace of the bench chunk's zlib stream as k_pinf_block / k_pinf_emit split it (tuning aid, not product code):
every Huffman block's body cut into L = min(1024, bits / 256) equal lanes, each lane starting at its first symbol
boundary at or past its share; per lane the symbols, literals, matches (short and >= 32 bytes, which
k_pinf_expand writes) and output bytes.  Prints, for the largest blocks, the lanes' maximum and mean of each, so
the slowest lane's work can be set against its measured time.
Usage: python tools/pinf_lane_sim.py [level] [kind: shuffled|ints|periodic]"""
import sys
import zlib

import numpy as np

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def chunk(kind):
    if kind == "shuffled":
        v = np.random.default_rng(0x5EED2000).standard_normal(1 << 20).astype(np.float32)
        return v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
    if kind == "ints":
        return np.random.default_rng(3).integers(-8, 9, 1 << 20).astype(np.float32).tobytes()
    return (np.arange(1 << 20) % 1000).astype(np.float32).tobytes()


class Bits:
    def __init__(self, data):
        self.v = int.from_bytes(data, "little")
        self.n = 8 * len(data)

    def get(self, p, n):
        return (self.v >> p) & ((1 << n) - 1)


def table(lens):
    """code (bit-reversed, as read LSB first) -> (symbol, length) for every code, keyed by (length, code)."""
    bl = [0] * 16
    for l in lens:
        bl[l] += 1
    bl[0] = 0
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, l in enumerate(lens):
        if l:
            c = nxt[l]
            nxt[l] += 1
            r = int(format(c, f"0{l}b")[::-1], 2)
            t[(l, r)] = s
    return t


def dec(B, p, t, maxlen=15):
    for l in range(1, maxlen + 1):
        s = t.get((l, B.get(p, l)))
        if s is not None:
            return s, l
    raise ValueError("bad code")


def trace(s):
    """yields (body_bit, end_bit, [(bit, bytes, kind)]) per Huffman block; kind 0 literal, 1 match, 2 eob"""
    B = Bits(s)
    p = 16   # zlib header
    blocks = []
    while True:
        final = B.get(p, 1)
        typ = B.get(p + 1, 2)
        p += 3
        if typ == 0:
            p = (p + 7) // 8 * 8
            ln = B.get(p, 16)
            p += 32 + 8 * ln
        else:
            if typ == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 30
            else:
                nl = B.get(p, 5) + 257
                nd = B.get(p + 5, 5) + 1
                nc = B.get(p + 10, 4) + 4
                p += 14
                cl = [0] * 19
                for i in range(nc):
                    cl[ORDER[i]] = B.get(p, 3)
                    p += 3
                ct = table(cl)
                lens = []
                while len(lens) < nl + nd:
                    sym, l = dec(B, p, ct, 7)
                    p += l
                    if sym < 16:
                        lens.append(sym)
                    elif sym == 16:
                        lens += [lens[-1]] * (3 + B.get(p, 2))
                        p += 2
                    elif sym == 17:
                        lens += [0] * (3 + B.get(p, 3))
                        p += 3
                    else:
                        lens += [0] * (11 + B.get(p, 7))
                        p += 7
                ll, dl = lens[:nl], lens[nl:]
            lt, dt = table(ll), table(dl)
            body = p
            syms = []
            while True:
                q = p
                sym, l = dec(B, p, lt)
                p += l
                if sym < 256:
                    syms.append((q, 1, 0))
                elif sym == 256:
                    syms.append((q, 0, 2))
                    break
                else:
                    k = sym - 257
                    ln = LBASE[k] + B.get(p, LEXT[k])
                    p += LEXT[k]
                    ds, l = dec(B, p, dt)
                    p += l + DEXT[ds]
                    syms.append((q, ln, 1))
            blocks.append((body, p, syms))
        if final:
            return blocks


def main():
    level = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    kind = sys.argv[2] if len(sys.argv) > 2 else "shuffled"
    s = zlib.compress(chunk(kind), level)
    blocks = trace(s)
    print(f"{kind} zlib-{level}: {len(s)} bytes, {len(blocks)} Huffman blocks")
    rows = []
    for body, end, syms in blocks:
        span = end - body
        L = max(1, min(1024, span // 256))
        bits = np.array([q for q, _, _ in syms], dtype=np.int64)
        lo = body + (span * np.arange(L + 1)) // L
        first = np.searchsorted(bits, lo[:-1])   # the lane's first symbol: at or past its share
        last = np.append(first[1:], len(syms))
        st = []
        for a, b in zip(first, last):
            seg = syms[a:b]
            lit = sum(1 for _, _, k in seg if k == 0)
            short = [n for _, n, k in seg if k == 1 and n < 32]
            long_ = [n for _, n, k in seg if k == 1 and n >= 32]
            st.append((len(seg), lit, len(short), len(long_), lit + sum(short), lit + sum(short) + sum(long_)))
        st = np.array(st)
        out = int(st[:, 5].sum())
        rows.append((out, span, L, st))
    rows.sort(key=lambda r: -r[0])
    print("out_bytes bits lanes | max/mean: symbols literals short_matches long_matches bytes_put bytes")
    for out, span, L, st in rows[:6]:
        mx, mean = st.max(axis=0), st.mean(axis=0)
        print(f"{out:8d} {span:7d} {L:5d} | " + "  ".join(f"{int(m)}/{a:.0f}" for m, a in zip(mx, mean)))
        k = int(np.argmax(st[:, 0] + st[:, 4]))
        print(f"{'':22s}   slowest lane by symbols + put bytes: {st[k].tolist()}")


if __name__ == "__main__":
    main()
