"""Which rounding model does v_mfma_f32_32x32x16_f16 follow?  Reads the probe's dump
(tools/probes/mfma_f16_probe.hip) and compares every GPU output with candidate models computed
exactly (Python integers, then round-to-nearest-even to float32):
  one      : rn32(C + sum_k a_k b_k)                      (exact sum, one rounding)
  seq      : t = C; t = rn32(t + a_k b_k) for k = 0..15
  sum_then : rn32(C + rn32(sum_k a_k b_k))
  pairs8   : rn32(C + rn32(S_0..7) + ...) two halves of 8, each exact, rounded, then added in order
  half_one : rn32(rn32(C + S_0..7) + S_8..15)             (two chained 8-term steps)
    python tools/probes/mfma_f16_models.py dump.bin
"""
import sys
from fractions import Fraction

import numpy as np

SC = 100  # integers in units of 2^-SC


def to_int(x):
    f = Fraction(float(x))
    v = f * (1 << SC)
    assert v.denominator == 1
    return int(v)


def rn32(n):
    """integer n (units of 2^-SC) rounded to the nearest float32 (ties to even), as a float."""
    if n == 0:
        return 0.0
    s = -1 if n < 0 else 1
    a = abs(n)
    e = a.bit_length()  # value in [2^(e-1), 2^e) units
    # float32 normal: 24 significant bits; exponent of the lsb = e - 24 (in units), clamp subnormals
    lsb = e - 24
    min_lsb = SC - 149  # 2^-149 in units of 2^-SC
    lsb = max(lsb, min_lsb)
    if lsb <= 0:
        return s * float(Fraction(a, 1 << SC))
    q, r = divmod(a, 1 << lsb)
    half = 1 << (lsb - 1)
    if r > half or (r == half and (q & 1)):
        q += 1
    return s * float(Fraction(q << lsb, 1 << SC))


def main():
    raw = open(sys.argv[1], "rb").read()
    nt = int(np.frombuffer(raw[:4], np.int32)[0])
    o = 4
    A = np.frombuffer(raw[o:o + nt * 512 * 2], np.float16).reshape(nt, 32, 16); o += nt * 512 * 2
    B = np.frombuffer(raw[o:o + nt * 512 * 2], np.float16).reshape(nt, 16, 32); o += nt * 512 * 2
    C = np.frombuffer(raw[o:o + nt * 1024 * 4], np.float32).reshape(nt, 32, 32); o += nt * 1024 * 4
    D = np.frombuffer(raw[o:o + nt * 1024 * 4], np.float32).reshape(nt, 32, 32)
    models = ["one", "seq", "sum_then", "pairs8", "half_one"]
    hits = {k: 0 for k in models}
    tot = 0
    rng = np.random.default_rng(0)
    for t in range(nt):
        for (i, j) in rng.integers(0, 32, size=(48, 2)):
            p = [to_int(float(A[t, i, k]) * float(B[t, k, j])) for k in range(16)]  # exact (22 bits)
            c = to_int(C[t, i, j])
            d = float(D[t, i, j])
            S = sum(p)
            got = {
                "one": rn32(c + S),
                "seq": None,
                "sum_then": rn32(c + to_int(rn32(S))),
                "pairs8": rn32(c + to_int(rn32(sum(p[:8]))) + to_int(rn32(sum(p[8:])))),
                "half_one": rn32(to_int(rn32(c + sum(p[:8]))) + sum(p[8:])),
            }
            x = c
            for k in range(16):
                x = to_int(rn32(x + p[k]))
            got["seq"] = float(Fraction(x, 1 << SC))
            for k in models:
                hits[k] += got[k] == d
            tot += 1
    print(f"{tot} outputs:", {k: f"{hits[k] / tot:.4f}" for k in models})


if __name__ == "__main__":
    main()
