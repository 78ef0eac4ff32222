import sys, numpy as np
sys.path.insert(0, '/root/repo')
from oracle import oracle as O
from cluster_tools_amd.synthetic import boundary_map
O.build()
cfg = dict(apply_dt_2d=True, apply_ws_2d=True)
x = boundary_map((2, 576, 576), seed=1, pitch=(3, 24, 24), origin=(64, 0, 0), full_shape=(256, 2048, 2048))
x = (x - x.min()); x = x / x.max()
sl = x[0]
fg = (sl > 0.5).astype(np.uint8)
dt = O.distance_transform(fg)
seeds = O.make_seeds(dt, dict(cfg, sigma_seeds=2.0))
hm = O.make_hmap(sl, dt, dict(cfg, sigma_weights=2.0, alpha=0.8))
Y, X = hm.shape
def ordf(f):
    u = f.view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)
H = ordf(hm.astype(np.float32))
INF = np.uint64(0xFFFFFFFFFFFFFFFF)
LM = np.uint64((1 << 20) - 1)
hp = np.pad(hm, 1, constant_values=np.inf)
nb = np.stack([hp[:-2, 1:-1], hp[2:, 1:-1], hp[1:-1, :-2], hp[1:-1, 2:]])
mn = nb.min(0); cnt = (nb == mn).sum(0)
par = np.arange(Y * X).reshape(Y, X); off = np.array([-X, X, -1, 1]); am = nb.argmin(0)
lower = (mn < hm) & (cnt == 1) & (seeds == 0)
p = np.where(lower, par + off[am], par).ravel()
for _ in range(25): p = p[p]
rs = seeds.ravel()[p]
fixed = (rs != 0).reshape(Y, X)
K = np.where(fixed, (H << np.uint64(32)) | rs.reshape(Y, X).astype(np.uint64), INF)
def f_packed(h, b):
    bh = b >> np.uint64(32); bl = b & np.uint64(0xFFFFFFFF)
    above = h > bh
    nh = np.maximum(h, bh)
    inc = bl + np.uint64(1 << 20)
    ovf = inc > np.uint64(0xFFFFFFFF)
    nl = np.where(above, bl & LM, np.where(ovf, bl, inc))
    return np.where(b == INF, INF, (nh << np.uint64(32)) | nl)
def nbmin(K):
    Kp = np.pad(K, 1, constant_values=INF)
    return np.minimum(np.minimum(Kp[:-2, 1:-1], Kp[2:, 1:-1]), np.minimum(Kp[1:-1, :-2], Kp[1:-1, 2:]))
# synchronous Jacobi iterations
Kj = K.copy(); it = 0
while True:
    nk = np.where(fixed, Kj, f_packed(H, nbmin(Kj)))
    it += 1
    if np.array_equal(nk, Kj): break
    Kj = nk
print('Jacobi iterations to converge:', it)
Kfinal = Kj
# per 64x64 chunk: Jacobi iterations with halo frozen at initial values (it0 local solve), then count
# how many voxels differ from the global fixpoint after local convergence
loc_it = []
wrong = 0
for cy in range(0, Y, 64):
    for cx in range(0, X, 64):
        y0, y1, x0, x1 = max(cy-1,0), min(cy+65,Y), max(cx-1,0), min(cx+65,X)
        sub = K[y0:y1, x0:x1].copy(); fx = fixed[y0:y1, x0:x1].copy()
        # halo cells frozen
        inner = np.zeros_like(fx); inner[cy-y0:cy-y0+64, cx-x0:cx-x0+64] = True
        frozen = fx | ~inner
        Hs = H[y0:y1, x0:x1]
        n = 0
        while True:
            nk = np.where(frozen, sub, f_packed(Hs, nbmin(sub)))
            n += 1
            if np.array_equal(nk, sub): break
            sub = nk
        loc_it.append(n)
        wrong += (sub[inner] != Kfinal[y0:y1, x0:x1][inner]).sum()
loc_it = np.array(loc_it)
print('local Jacobi iterations per chunk: mean %.1f pct90 %d max %d; voxels still wrong after local solve %.3f of open' % (loc_it.mean(), np.percentile(loc_it, 90), loc_it.max(), wrong / (~fixed).sum()))
# Gauss-Seidel fast sweeping: 4 sweep directions (rows down/up, cols right/left), count rounds
def sweep_rows(K, rev):
    rng = range(Y - 1, -1, -1) if rev else range(Y)
    ch = False
    for y in rng:
        Kp = np.pad(K, 1, constant_values=INF)
        m = np.minimum(np.minimum(Kp[y, 1:-1], Kp[y + 2, 1:-1]), np.minimum(Kp[y + 1, :-2], Kp[y + 1, 2:]))
        nk = np.where(fixed[y], K[y], f_packed(H[y], m))
        if not np.array_equal(nk, K[y]): ch = True
        K[y] = nk
    return ch
Kg = K.copy(); rounds = 0
while True:
    rounds += 1
    c = sweep_rows(Kg, False); c |= sweep_rows(Kg, True)
    Kt = Kg.T.copy(); fixed_t = fixed; 
    # columns: transpose
    Kg2 = Kg.T.copy(); fixed, H, Y, X = fixed.T.copy(), H.T.copy(), X, Y
    c |= sweep_rows(Kg2, False); c |= sweep_rows(Kg2, True)
    Kg = Kg2.T.copy(); fixed, H, Y, X = fixed.T.copy(), H.T.copy(), X, Y
    if not c: break
print('fast sweeping rounds (row down/up + col right/left, whole slice):', rounds, 'equal to Jacobi fixpoint:', np.array_equal(Kg, Kfinal))
