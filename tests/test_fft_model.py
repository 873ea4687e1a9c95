"""Host model of the front end's four-step FFT index math (csrc/frontend.hip,
fe_mel_db_kernel): 64 lanes x 16 registers, dft16 with its output permutation
fe_p16, the per-lane twiddles W1024^{l k1}, the XOR-swizzled transpose
(k1*64 + (l ^ 4 k1)), the second dft16 over s (lane (g, q) holds B[q + 4s][g]),
W64^{q k2}, the radix-4 across each lane quad (partners q^2 then q^1, the -i on
q = 3) and the padded scatter fe_zslot(g + 16 k2 + 256 br(q)).  Compared with
numpy's FFT in float64: any index slip shows up as an O(1) error."""
import numpy as np

N = 1024


def _w(n, k):
    return np.exp(-2j * np.pi * k / n)


def _p16(k):
    return 4 * (k & 3) + (k >> 2)


def _dft4(a, b, c, d):
    s02, d02, s13, d13 = a + c, a - c, b + d, b - d
    return s02 + s13, d02 - 1j * d13, s02 - s13, d02 + 1j * d13


def _dft16(x):
    x = list(x)
    for t2 in range(4):
        x[t2], x[4 + t2], x[8 + t2], x[12 + t2] = _dft4(x[t2], x[4 + t2], x[8 + t2], x[12 + t2])
    for k1 in range(1, 4):
        for t2 in range(1, 4):
            x[4 * k1 + t2] *= _w(16, t2 * k1)
    for k1 in range(4):
        x[4 * k1:4 * k1 + 4] = _dft4(*x[4 * k1:4 * k1 + 4])
    return x


def _zslot(k):
    return k + 4 * (k >> 8)


def four_step(z):
    buf = np.zeros(N + 16, complex)
    for lane in range(64):
        X = _dft16([z[lane + 64 * t] for t in range(16)])
        for k1 in range(1, 16):
            X[_p16(k1)] *= _w(N, lane * k1)
        for k1 in range(16):
            buf[k1 * 64 + (lane ^ (4 * k1))] = X[_p16(k1)]
    D = []
    for lane in range(64):
        g, q = lane >> 2, lane & 3
        Y = _dft16([buf[g * 64 + ((q + 4 * s) ^ (4 * g))] for s in range(16)])
        D.append([Y[_p16(k2)] * _w(64, q * k2) for k2 in range(16)])

    def stage1(lane, k2):
        q = lane & 3
        d, p = D[lane][k2], D[lane ^ 2][k2]
        u = d + p if q < 2 else p - d
        return u * -1j if q == 3 else u

    out = np.zeros(N + 16, complex)
    br = {0: 0, 1: 2, 2: 1, 3: 3}
    for lane in range(64):
        g, q = lane >> 2, lane & 3
        for k2 in range(16):
            u, u2 = stage1(lane, k2), stage1(lane ^ 1, k2)
            out[_zslot(g + 16 * k2 + 256 * br[q])] = u + u2 if (q & 1) == 0 else u2 - u
    return np.array([out[_zslot(k)] for k in range(N)])


def test_dft16_permutation():
    v = np.random.default_rng(1).standard_normal(16) + 0j
    X = _dft16(v)
    assert np.allclose([X[_p16(k)] for k in range(16)], np.fft.fft(v))


def test_four_step_matches_fft():
    rng = np.random.default_rng(0)
    z = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    assert np.abs(four_step(z) - np.fft.fft(z)).max() < 1e-9


def test_transpose_and_scatter_are_bank_conflict_free():
    # transpose read: lanes of a 32-lane group hit 64 distinct dword banks (b64)
    for s in range(16):
        for half in (0, 32):
            banks = set()
            for lane in range(half, half + 32):
                g, q = lane >> 2, lane & 3
                a = 2 * (g * 64 + ((q + 4 * s) ^ (4 * g)))
                banks |= {a % 64, (a + 1) % 64}
            assert len(banks) == 64
    # spectrum scatter (b64 write, 16-lane groups, bank mod 32)
    for k2 in range(16):
        for g0 in range(0, 64, 16):
            banks = set()
            for lane in range(g0, g0 + 16):
                g, q = lane >> 2, lane & 3
                a = 2 * _zslot(g + 16 * k2 + 256 * {0: 0, 1: 2, 2: 1, 3: 3}[q])
                banks |= {a % 32, (a + 1) % 32}
            assert len(banks) == 32
