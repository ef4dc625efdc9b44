"""k_pinf_find lists a dynamic-block header only when its code-length symbols follow the run-length coding of
zlib's encoder (k_pinflate.hip `rle_impossible`: no third explicit zero, no zero run continued after a 17, no
17 / 18 after an explicit zero, no 16 repeating a zero, no fourth explicit repeat of a length within one code).  Real zlib / GNU gzip streams must never break those
rules, or their blocks would reach the chain as misses (correct, but decoded by the host).  This parses every
dynamic header of real streams — CPython's zlib (the C library) at every level, strategy and memLevel over
several data kinds, and GNU gzip when installed — and checks the rules on each.  (The rules are the encoder's
property, not RFC 1951's: the block parse, k_pinf_block, accepts any valid header.)"""
import shutil
import subprocess
import zlib

import numpy as np
import pytest

ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DEXT = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]


def rle_impossible(sym, psym, z0, prev, same, first_dist):   # the device rule, restated
    return ((sym == 0 and psym == 0 and z0 >= 2) or (psym == 17 and (sym == 0 or sym >= 16))
            or (psym == 0 and sym >= 17) or (sym == 16 and prev == 0)
            or (1 <= sym <= 15 and sym == psym and same >= 2 and not first_dist))


def rle_same(sym, psym, same, first_dist):
    return same + 1 if 1 <= sym <= 15 and sym == psym and not first_dist else 0


class Reader:
    def __init__(self, data):
        self.v = int.from_bytes(data, "little")

    def get(self, p, n):
        return (self.v >> p) & ((1 << n) - 1)


def table(lens):
    bl = [0] * 16
    for ln in lens:
        bl[ln] += 1
    bl[0] = 0
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, ln in enumerate(lens):
        if ln:
            c = nxt[ln]
            nxt[ln] += 1
            t[(ln, int(format(c, f"0{ln}b")[::-1], 2))] = s
    return t


def dec(r, p, t):
    for ln in range(1, 16):
        s = t.get((ln, r.get(p, ln)))
        if s is not None:
            return s, ln
    raise ValueError("bad code")


def header_symbol_runs(raw):
    """every dynamic block's code-length symbols (a raw DEFLATE stream)"""
    r = Reader(raw)
    p, out = 0, []
    while True:
        final, typ = r.get(p, 1), r.get(p + 1, 2)
        p += 3
        if typ == 0:
            p = (p + 7) // 8 * 8
            p += 32 + 8 * r.get(p, 16)
        else:
            if typ == 1:
                ll, dl = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8, [5] * 30
            else:
                nl, nd, nc = r.get(p, 5) + 257, r.get(p + 5, 5) + 1, r.get(p + 10, 4) + 4
                p += 14
                cl = [0] * 19
                for i in range(nc):
                    cl[ORDER[i]] = r.get(p, 3)
                    p += 3
                ct, lens, syms = table(cl), [], []
                while len(lens) < nl + nd:
                    sym, ln = dec(r, p, ct)
                    p += ln
                    syms.append((sym, lens[-1] if lens else 0, len(lens) == nl))
                    if sym < 16:
                        lens.append(sym)
                    elif sym == 16:
                        lens += [lens[-1]] * (3 + r.get(p, 2))
                        p += 2
                    elif sym == 17:
                        lens += [0] * (3 + r.get(p, 3))
                        p += 3
                    else:
                        lens += [0] * (11 + r.get(p, 7))
                        p += 7
                out.append(syms)
                ll, dl = lens[:nl], lens[nl:]
            lt, dt = table(ll), table(dl)
            while True:
                sym, ln = dec(r, p, lt)
                p += ln
                if sym == 256:
                    break
                if sym > 256:
                    p += LEXT[sym - 257]
                    ds, ln = dec(r, p, dt)
                    p += ln + DEXT[ds]
        if final:
            return out


def check(raw):
    runs = header_symbol_runs(raw)
    for syms in runs:
        psym, z0, same = 19, 0, 0
        for sym, prev, first_dist in syms:
            assert not rle_impossible(sym, psym, z0, prev, same, first_dist), (sym, psym, z0, prev, same)
            same = rle_same(sym, psym, same, first_dist)
            z0 = z0 + 1 if sym == 0 else 0
            psym = sym
    return len(runs)


def kinds():
    rng = np.random.default_rng(11)
    v = rng.standard_normal(4096).astype(np.float32)
    yield "shuffled_f32", v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
    yield "ints_f32", rng.integers(-8, 9, 4096).astype(np.float32).tobytes()
    yield "i64_small", rng.integers(0, 300, 2048).astype(np.int64).tobytes()
    yield "text", b" ".join(b"w%d" % int(x) for x in rng.zipf(1.3, 3000))[:16384]
    yield "skewed_bytes", rng.geometric(0.05, 16384).clip(0, 255).astype(np.uint8).tobytes()


@pytest.mark.parametrize("strategy", [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE])
def test_zlib_headers_follow_the_finders_rules(strategy):
    n = 0
    for _, raw in kinds():
        for level in (1, 6, 9):
            for mem in (8, 9):
                c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
                n += check(c.compress(raw) + c.flush())
    assert n > 0


@pytest.mark.skipif(shutil.which("gzip") is None, reason="GNU gzip not installed")
def test_gnu_gzip_headers_follow_the_finders_rules():
    n = 0
    for _, raw in kinds():
        for level in ("-1", "-6", "-9"):
            gz = subprocess.run(["gzip", "-c", "-n", level], input=raw, capture_output=True, check=True).stdout
            n += check(gz[10:-8])   # (no FNAME with -n: a 10-byte header)
    assert n > 0


def test_rules_reject_what_they_should():
    # a third explicit zero, a 17 continued by a zero, 18 after an explicit zero, 16 repeating a zero, a fourth
    # explicit repeat of a length (but not across the literal / distance boundary)
    assert rle_impossible(0, 0, 2, 0, 0, False)
    assert rle_impossible(0, 17, 0, 0, 0, False) and rle_impossible(18, 17, 0, 0, 0, False)
    assert rle_impossible(17, 0, 1, 0, 0, False)
    assert rle_impossible(16, 18, 0, 0, 0, False)
    assert rle_impossible(7, 7, 0, 7, 2, False) and not rle_impossible(7, 7, 0, 7, 2, True)
    assert not rle_impossible(7, 7, 0, 7, 1, False)
    assert not rle_impossible(0, 18, 0, 0, 0, False) and not rle_impossible(17, 18, 0, 0, 0, False)
    assert not rle_impossible(5, 17, 0, 0, 0, False)
