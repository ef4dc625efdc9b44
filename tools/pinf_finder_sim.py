"""CPU simulation of k_pinf_find's survivor header test for one workgroup's 8 KiB of the bench chunk's zlib-1 stream
(tuning aid, not product code): every bit offset screened as the finder does (BTYPE 2, HLIT / HDIST, a complete
code-length code), then each survivor's code lengths decoded until rejected, printing the survivors' longest
decodes (iterations = code-length symbols).  Usage: python tools/pinf_finder_sim.py [workgroup]"""
import os, zlib, numpy as np, sys
RLE = os.environ.get("RLE", "0") == "1"
RLE4 = os.environ.get("RLE4", "0") == "1"   # also: no fourth explicit repeat of a nonzero length   # the finder's run-length rules (k_pinflate.hip rle_impossible)
rng = np.random.default_rng(0x5EED2000)
v = rng.standard_normal(1 << 20).astype(np.float32)
sh = v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
s = zlib.compress(sh, 1)
data = np.frombuffer(s + bytes(64), dtype=np.uint8)
bits = np.unpackbits(data, bitorder='little')
def getbits(p, n):
    v = 0
    for i in range(n): v |= int(bits[p + i]) << i
    return v
ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
def decode_header(p, end_bits):
    h = getbits(p, 17)
    if ((h >> 1) & 3) != 2 or ((h >> 3) & 31) > 29 or ((h >> 8) & 31) > 29: return None
    nl = ((h >> 3) & 31) + 257; nd = ((h >> 8) & 31) + 1; nc = ((h >> 13) & 15) + 4
    lens = [0] * 19
    for i in range(nc): lens[ORDER[i]] = getbits(p + 17 + 3 * i, 3)
    # complete code?
    cnt = [0] * 8
    for l in lens: cnt[l] += 1
    left = 1
    for l in range(1, 8):
        left = (left << 1) - cnt[l]
        if left < 0: return ('over', 0)
    if left != 0: return ('incomplete', 0)
    # canonical codes
    code = 0; nxt = [0] * 9
    for b in range(1, 8):
        code = (code + cnt[b - 1] * (b > 1)) << 1 if b > 1 else 0
        nxt[b] = code
    # build decode map: (len, code msb-first) -> sym
    codes = {}
    c = 0; bl = [0]*8
    cnt0 = cnt[:]; cnt0[0] = 0
    code = 0; next_code = [0]*9
    for b in range(1, 8):
        code = (code + cnt0[b - 1]) << 1
        next_code[b] = code
    for sym in range(19):
        l = lens[sym]
        if l:
            codes[(l, next_code[l])] = sym; next_code[l] += 1
    pos = p + 17 + 3 * nc
    total = nl + nd; idx = 0; prev = 0; kl = kd = 0; it = 0; psym = 19; z0 = 0; same = 0
    while idx < total:
        it += 1
        # decode one symbol msb-first
        cv = 0; sym = None
        for l in range(1, 8):
            cv = (cv << 1) | int(bits[pos + l - 1])
            if (l, cv) in codes: sym = codes[(l, cv)]; used = l; break
        if sym is None: return ('nosym', it)
        pos += used
        if RLE and ((sym == 0 and psym == 0 and z0 >= 2) or (psym == 17 and (sym == 0 or sym >= 16))
                    or (psym == 0 and sym >= 17) or (sym == 16 and prev == 0)):
            return ('rle', it)
        if RLE4 and 1 <= sym <= 15 and sym == psym and same >= 2:
            return ('rle4', it)
        same = same + 1 if (1 <= sym <= 15 and sym == psym) else 0
        z0 = z0 + 1 if sym == 0 else 0
        psym = sym
        if sym == 16:
            if idx == 0: return ('rep0', it)
            rep = 3 + getbits(pos, 2); pos += 2; val = prev
        elif sym == 17: rep = 3 + getbits(pos, 3); pos += 3; val = 0
        elif sym == 18: rep = 11 + getbits(pos, 7); pos += 7; val = 0
        else: rep = 1; val = sym
        if idx + rep > total: return ('overrun', it)
        nlit = min(rep, max(0, nl - idx)); ndst = rep - nlit
        if val:
            kl += nlit << (15 - val); kd += ndst << (15 - val)
            if kl > 1 << 15 or kd > 1 << 15: return ('oversub', it)
        idx += rep; prev = val
        if pos > end_bits: return ('end', it)
    return ('ok' if kl == 1 << 15 else 'inc', it)
wg = int(sys.argv[1]) if len(sys.argv) > 1 else 306
q0 = wg * 8192
res = []
for byte in range(q0, min(q0 + 8192, len(s))):
    for b in range(8):
        r = decode_header(8 * byte + b, 8 * len(s))
        if r is not None and r[0] not in ('over', 'incomplete'): res.append((8 * byte + b, r))
its = sorted((r[1], r[0], p) for p, r in res)
print("stream", len(s), "wg", wg, "rle", RLE, "survivors", len(res), "max iterations", its[-5:],
      "alive past 16/32/64/96:", [sum(1 for r in res if r[1][1] > k) for k in (16, 32, 64, 96)])
