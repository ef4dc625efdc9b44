"""Device blosc2 decode timing (k_blosc2): a batch of 4 MiB f32 chunks and a lone chunk per call, for
both LZ codecs and a few block sizes.  One JSON line per case.
    python tools/probe_blosc2.py [n_chunks] [codec,codec,...]   (lz4 blosclz zstd lz4_lib; zstd / lz4_lib: streams
    by the real libzstd / liblz4 through pyarrow)"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "reductionist-rs_amd"), str(ROOT)):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from datagen import blosc2_chunk as B  # noqa: E402
from reductionist_amd import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    eng = Engine([0])
    ws = eng.workspace(0)
    rng = np.random.default_rng(1)
    elems = 1 << 20
    raw_len = 4 * elems
    raws = [(np.round(np.cumsum(rng.standard_normal(elems)) * 64) / 64).astype(np.float32).tobytes() for _ in range(8)]
    d_out = torch.empty(n * raw_len, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_err = torch.zeros(n, dtype=torch.int32, device="cuda")
    want = sys.argv[2].split(",") if len(sys.argv) > 2 else ["lz4", "blosclz"]
    codecs = {"lz4": (B.LZ4, "repo"), "blosclz": (B.BLOSCLZ, "repo"), "zstd": (B.ZSTD, "lib"), "lz4_lib": (B.LZ4, "lib")}
    for name in want:
        codec, enc = codecs[name]
        for bs in (1 << 15, 1 << 16, 1 << 18):
            chunks = [B.build(r, 4, bs, codec, (0, 0, 0, 0, 0, B.SHUFFLE), memcpyed=False, enc=enc) for r in raws]
            offs, total = [], 0
            for c in chunks:
                offs.append(total)
                total += (len(c) + 255) // 256 * 256
            host = np.zeros(total, dtype=np.uint8)
            for o, c in zip(offs, chunks):
                host[o:o + len(c)] = np.frombuffer(c, dtype=np.uint8)
            d_in = torch.from_numpy(host).cuda()
            ptrs = [d_in.data_ptr() + offs[i % 8] for i in range(n)]
            lens = [len(chunks[i % 8]) for i in range(n)]

            def run(k):
                ws.decompress_batch_device("blosc2", ptrs[:k], lens[:k], d_out.data_ptr(), raw_len, d_len.data_ptr(),
                                           d_err.data_ptr(), None)

            res = {"codec": name, "block": bs, "ratio": round(raw_len * 8 / sum(len(c) for c in chunks), 3)}
            for k, reps in ((n, 3), (1, 10)):
                run(k)
                torch.cuda.synchronize()
                assert int(d_err[:k].abs().sum()) == 0
                assert d_out[:raw_len].cpu().numpy().tobytes() == raws[0]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(k)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 1e3 / reps
                res[f"n{k}_ms"] = round(t * 1e3, 3)
                res[f"n{k}_GBs"] = round(k * raw_len / t / 1e9, 2)
            print(json.dumps(res), flush=True)
    ws.close()
    eng.close()


if __name__ == "__main__":
    main()
