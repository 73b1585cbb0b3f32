"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (CPU only):  python tests/golden/make_golden.py

Sources of truth:
* upstream_kat.json -- known-answer tests published in the test suite of the
  upstream crate reed-solomon-erasure (galois_8 mul/exp/div KATs, matrix
  multiply/inverse KATs, RS(5,5) "one encode"). These are literal facts of
  the upstream suite, entered here as data; the reference (helyim) has no EC
  tests of its own. The oracle must reproduce them.
* every other file is OUTPUT of oracle/rs_oracle.py (numpy restatement),
  cross-checked at generation time against oracle/rs_oracle.c.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import rs_oracle as O  # noqa: E402
from oracle import corc  # noqa: E402

UPSTREAM_KAT = {
    "gf_mul": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
    "gf_div": [[0, 7, 0], [3, 3, 1], [6, 3, 2]],
    "gf_exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
    "matrix_mul": {"a": [[1, 2], [3, 4]], "b": [[5, 6], [7, 8]], "out": [[11, 22], [19, 42]]},
    "matrix_inverse": [
        {"m": [[56, 23, 98], [3, 100, 200], [45, 201, 123]],
         "inv": [[175, 133, 33], [130, 13, 245], [112, 35, 126]]},
        {"m": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 0, 1, 0], [0, 0, 0, 0, 1], [7, 7, 6, 6, 1]],
         "inv": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [123, 123, 1, 122, 122], [0, 0, 1, 0, 0],
                 [0, 0, 0, 1, 0]]},
    ],
    "rs_5_5_one_encode": {
        "data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
        "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]],
    },
    "rs_10_4_parity_rows": [
        [0x81, 0x96, 0xaf, 0xb8, 0xd2, 0xc4, 0xfe, 0xe8, 0x03, 0x02],
        [0x96, 0x81, 0xb8, 0xaf, 0xc4, 0xd2, 0xe8, 0xfe, 0x02, 0x03],
        [0xbf, 0xd6, 0x62, 0x0a, 0x06, 0x6f, 0xdf, 0xb7, 0x05, 0x04],
        [0xd6, 0xbf, 0x0a, 0x62, 0x6f, 0x06, 0xb7, 0xdf, 0x04, 0x05],
    ],
}

ENCODE_LENGTHS = [1, 3, 15, 16, 17, 64, 255, 4097, 65536, 1 << 20]
DECODE_PATTERNS = [[0, 5, 10, 13], [0, 1, 2, 3], [10, 11, 12, 13], [6, 7, 8, 9], [9], [13],
                   [0, 13], [3, 4, 11], [1, 2, 3, 4], [4, 5, 6, 7], [2, 9, 10, 12]]
VOLUME_BYTES = 30_000_000
VOLUME_DROPS = [[0, 5, 10, 13], [0, 1, 2, 3], [10, 11, 12, 13], [6, 7, 8, 9]]


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


def main():
    dump("upstream_kat.json", UPSTREAM_KAT)

    rs = O.ReedSolomon(10, 4)
    crs = corc.CReedSolomon(10, 4)
    assert np.array_equal(rs.matrix, crs.matrix())
    dump("tables.json", {
        "exp_sha256": O.sha256(O.EXP_TABLE[:255]),
        "log_sha256": O.sha256(O.LOG_TABLE[1:].astype(np.uint8)),
        "mul_sha256": O.sha256(O.MUL_TABLE),
        "matrix_10_4": rs.matrix.tolist(),
    })

    # encode vectors: stripe s=0 of splitmix64(0x5EED0000 + s), parity sha256 per shard
    enc = {}
    for L in ENCODE_LENGTHS:
        data = O.stripe_data(0, L)
        shards = [data[i].copy() for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        rs.encode(shards)
        cshards = [data[i].copy() for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        crs.encode(cshards)
        for j in range(4):
            assert np.array_equal(shards[10 + j], cshards[10 + j]), (L, j)
        ent = {"data_sha256": O.sha256(data), "parity_sha256": [O.sha256(shards[10 + j]) for j in range(4)]}
        if L <= 64:
            ent["data_hex"] = [data[i].tobytes().hex() for i in range(10)]
            ent["parity_hex"] = [shards[10 + j].tobytes().hex() for j in range(4)]
        enc[str(L)] = ent
    dump("encode_vectors.json", {"seed": O.STRIPE_SEED_BASE, "stripe": 0, "vectors": enc})

    # decode matrices (inverse of the first-10-present sub-matrix) per pattern
    dec = {}
    for pat in DECODE_PATTERNS:
        present = [i for i in range(14) if i not in pat]
        valid = present[:10]
        inv = O.mat_invert(rs.matrix[valid, :])
        dec[",".join(map(str, pat))] = {"valid": valid, "inverse": inv.tolist()}
    dump("decode_matrices.json", dec)

    # 30 MB synthetic volume -> 14 shard files, drop 4 -> rebuild
    vol = O.synthetic_volume(VOLUME_BYTES)
    with tempfile.TemporaryDirectory() as td:
        base = os.path.join(td, "1")
        with open(base + ".dat", "wb") as f:
            f.write(vol.tobytes())
        O.write_ec_files(base)
        shas = []
        sizes = []
        for i in range(14):
            b = open(base + O.to_ext(i), "rb").read()
            shas.append(O.sha256(b))
            sizes.append(len(b))
        for drop in VOLUME_DROPS:
            for i in drop:
                os.remove(base + O.to_ext(i))
            rebuilt = O.rebuild_ec_files(base)
            assert rebuilt == sorted(drop), rebuilt
            for i in drop:
                assert O.sha256(open(base + O.to_ext(i), "rb").read()) == shas[i]
    dump("volume_30mb.json", {
        "dat_bytes": VOLUME_BYTES, "dat_sha256": O.sha256(vol), "volume_seed": O.VOLUME_SEED,
        "shard_sha256": shas, "shard_bytes": sizes, "drops": VOLUME_DROPS,
    })
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
