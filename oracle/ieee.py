"""Exact fp32 arithmetic helpers for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/.  Nothing here is on the product path.

The reference runs on CPU ATen (torch 2.10.0).  Its decision path is made of
IEEE fp32 operations in a fixed order; numpy reproduces every correctly rounded
fp32 op (+ - * / sqrt) exactly.  Two more primitives are needed:

* fma32      - fused multiply-add, rounded once (oneDNN conv / MKL sgemm
               accumulate with FMA).
* aten_sum   - ATen's CPU cascade outer-reduction order
               (aten/src/ATen/native/cpu/SumKernel.cpp: vectorized_outer_sum /
               multi_row_sum / row_sum), pinned against torch in
               tests/test_oracle_cpu.py.
* cr32       - a transcendental evaluated in float64 and rounded once to fp32,
               i.e. the correctly rounded fp32 result (the HIP kernels evaluate
               the same functions in double precision and round once).
"""
import numpy as np

f32 = np.float32
f64 = np.float64

# ATen's vectorized_outer_sum handles columns in blocks of 4 x Vectorized<float>
# = 32 columns on this build; trailing columns use row_sum's 4-way interleave.
ATEN_COL_BLOCK = 32


def fma32(a, b, c):
    """Correctly rounded fp32 fma(a, b, c) (vectorized, exact).

    a*b is exact in float64; the float64 sum is rounded once and then again to
    fp32.  Double rounding can only err when the float64 sum lands exactly on
    an fp32 midpoint while the exact sum did not; the exact residual of the
    float64 addition (TwoSum) decides that case.
    """
    a = np.asarray(a, f32).astype(f64)
    b = np.asarray(b, f32).astype(f64)
    c = np.asarray(c, f32).astype(f64)
    p = a * b
    s = p + c
    bb = s - p
    e = (p - (s - bb)) + (c - bb)
    r = s.astype(f32)
    rd = r.astype(f64)
    up = np.nextafter(r, f32(np.inf))
    dn = np.nextafter(r, f32(-np.inf))
    nb = np.where(s > rd, up, dn)
    mid = (rd + nb.astype(f64)) * 0.5
    tie = (s == mid) & (e != 0) & (s != rd)
    if np.any(tie):
        hi = np.maximum(r, nb)
        lo = np.minimum(r, nb)
        r = np.where(tie, np.where(e > 0, hi, lo), r)
    return r.astype(f32)


def cr32(fn, *args):
    """Correctly rounded fp32 value of a float64 libm function of fp32 args."""
    return np.asarray(fn(*[np.asarray(a, f32).astype(f64) for a in args])).astype(f32)


def _ceil_log2(n):
    return 1 if n <= 2 else int(n - 1).bit_length()


def _cascade(rows):
    """multi_row_sum: rows (n, ...) fp32 -> sum over axis 0 in ATen cascade order."""
    n = rows.shape[0]
    shape = rows.shape[1:]
    lp = max(4, _ceil_log2(n) // 4)
    step = 1 << lp
    mask = step - 1
    acc = np.zeros((4,) + shape, f32)
    i = 0
    while i + step <= n:
        for _ in range(step):
            acc[0] = acc[0] + rows[i]
            i += 1
        for j in range(1, 4):
            acc[j] = acc[j] + acc[j - 1]
            acc[j - 1] = 0
            if i & (mask << (j * lp)):
                break
    while i < n:
        acc[0] = acc[0] + rows[i]
        i += 1
    return ((acc[0] + acc[1]) + acc[2]) + acc[3]


def _rowsum(rows):
    """row_sum: 4 interleaved cascade partials, leftovers into partial 0."""
    n = rows.shape[0]
    nilp = n // 4
    parts = [_cascade(rows[k:4 * nilp:4]) for k in range(4)]
    p0 = parts[0]
    for i in range(4 * nilp, n):
        p0 = p0 + rows[i]
    return ((p0 + parts[1]) + parts[2]) + parts[3]


def aten_sum(rows, col_offset=0, ncols_total=None):
    """Sum rows (n, M) fp32 over axis 0 as ATen's contiguous outer reduction does.

    Columns with global index >= floor(ncols_total/32)*32 use the row_sum
    (tail) order, the others the vectorized cascade.  `col_offset` /
    `ncols_total` place this block of columns inside the full reduction.
    """
    rows = np.asarray(rows, f32)
    M = rows.shape[1]
    if ncols_total is None:
        ncols_total = M
    cut = (ncols_total // ATEN_COL_BLOCK) * ATEN_COL_BLOCK
    out = _cascade(rows).astype(f32)
    gidx = col_offset + np.arange(M)
    tail = gidx >= cut
    if np.any(tail):
        out[tail] = _rowsum(rows[:, tail])
    return out


def seq_sum(rows):
    """Plain sequential fp32 sum over axis 0 starting from 0."""
    acc = np.zeros(rows.shape[1:], f32)
    for r in rows:
        acc = acc + r
    return acc


def rint32(v):
    """torch.round: round half to even."""
    return np.rint(np.asarray(v, f32)).astype(f32)


def sleef_expf32(d):
    """SLEEF expf_u10 as libtorch_cpu's AVX-512 build evaluates it (the exp of
    ATen's vectorized float kernels): q = rint(d * log2(e)), two-FMA Cody-Waite
    reduction, degree-6 FMA polynomial, 1 + s*s*u + s, scaled by 2^(q>>1) and
    2^(q - q>>1).  Constants read from the libtorch_cpu.so that generated the
    golden fixtures."""
    d = np.asarray(d, f32)
    qf = np.rint((d * f32(1.44269502162933349609375)).astype(f32)).astype(f32)
    q = qf.astype(np.int64)
    s = fma32(qf, f32(-0.693145751953125), d)
    s = fma32(qf, f32(-1.428606765330187045e-06), s)
    u = np.full(d.shape, f32(0.000198527617612853646278381), f32)
    for c in (0.00139304355252534151077271, 0.00833336077630519866943359, 0.0416664853692054748535156,
              0.166666671633720397949219, 0.5):
        u = fma32(u, s, f32(c))
    u = (f32(1.0) + fma32((s * s).astype(f32), u, s)).astype(f32)
    a = q >> 1
    b = q - a
    u = (u * ((a + 127).astype(np.uint32) << 23).view(f32)).astype(f32)
    u = (u * ((b + 127).astype(np.uint32) << 23).view(f32)).astype(f32)
    u = np.where(d < f32(-104.0), f32(0.0), u)
    return np.where(d > f32(100.0), f32(np.inf), u).astype(f32)


def aten_softmax_vec_lanes(B, NT, threads, batch_offset=0, batch_total=None):
    """(B, NT) bool: True where ATen's dim-1 softmax of a (batch_total, 2, ht, wt)
    tensor evaluates exp vectorized (SLEEF), False where the scalar tail (glibc
    expf, correctly rounded) does.  at::parallel_for cuts the flattened
    (image, tile) range into ceil(N / T) chunks; inside a chunk each image's
    run is vectorized 16 lanes at a time and its last < 16 positions are
    scalar.  Checked against torch.softmax for T = 1..16 (tests/test_oracle_cpu.py)."""
    bt = B if batch_total is None else batch_total
    N = bt * NT
    nthr = max(1, min(int(threads), N))
    chunk = -(-N // nthr)
    lanes = np.zeros(N, bool)
    for cs in range(0, N, chunk):
        ce = min(N, cs + chunk)
        img = cs // NT
        while img * NT < ce:
            ss, se = max(cs, img * NT), min(ce, (img + 1) * NT)
            lanes[ss:ss + ((se - ss) // 16) * 16] = True
            img += 1
    return lanes[batch_offset * NT:(batch_offset + B) * NT].reshape(B, NT)
