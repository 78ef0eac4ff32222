// k_basin.hip — the flood's open voxels solved on the catchment graph ("basin flood").
//
// Reference: utils/volume_utils.py:123-128 (vu.watershed -> vigra.analysis.watershedsNew).  The
// flood's result is the fixpoint of k_flood.hip's header,
//     K(q) = f_q(min_p K(p)),   f_q(C, d) = h(q) > C ? (h(q), 0) : (C, d + 1),
//     label(q) = label(argmin_p (K(p), label(p))),
// with the packed key (C | d | label).  After the descent (k_descent_tile / k_descent_init) a
// voxel is final (its steepest descent reaches a seed) or open; an open voxel q descends strictly
// to a root r(q) without a seed (a local minimum of h, or a voxel whose lowest neighbour height is
// tied).  The frontier relaxation visits each open voxel ~5 times (it floods a catchment first
// through whatever pass it meets, then again through the lowest one).  Here:
//
// 1. C(q) = max(h(q), C(r(q))).  The descent path q -> r(q) never rises above h(q), so
//    C(q) <= max(h(q), C(r)); a path from the seeds to q continued down to r gives
//    C(r) <= max(C(q), h(q)) = C(q).
// 2. C(r) on the catchment graph.  Its nodes are the catchments {q : r(q) = r}, its sources the
//    final voxels: C(r_A) = min(min over neighbour pairs (q in A, p final) of max(h(q), h(p)),
//    min over pairs (q in A, p in B) of max(h(q), h(p), C(r_B))) -- crossing a catchment from an
//    entry to an exit costs no more than the two heights (down to the root and up again), so the
//    minimax paths between catchments are the minimax paths of the voxel graph.
//    k_basin_edges reduces the pairs over runs of lanes (atomicMin on the root's C for final
//    neighbours, an edge list for catchment pairs); k_basin_relax is Bellman-Ford on the list
//    (config 3: ~1.5 % of the open voxels become edges, 2 sweeps to converge).
// 3. d.  q with h(q) > min_p C(p) has d = 0 and C(q) = h(q).  The others (lake voxels: a few per
//    cent of the open voxels) have C(q) = min_p C(p); their d comes from the frontier relaxation
//    restricted to them, with every other key final in (C, d) (k_basin_keys).
// 4. labels.  With (C, d) known everywhere, an open voxel's parent is its argmin (C, d)
//    neighbour.  k_basin_tile resolves the parent chains inside 64 x 64 (2-D) / 16^3 tiles by
//    pointer jumping in LDS, as k_descent_tile; k_basin_hop follows them across tiles.  A voxel
//    with two argmin neighbours takes the first; the fixpoint takes the smaller of their labels,
//    so its label is an upper bound (as is every label below it).  k_flood_verify then marks
//    each voxel whose key is not f(min of its neighbours), and the frontier relaxation repairs
//    from there: Bellman-Ford from keys that are all keys of actual paths.
// Only the schedule differs from the frontier relaxation: the result is the same unique
// fixpoint, and k_flood_verify checks it as before.
#include "ctws_kernels.h"

namespace ctws {

// catchment root (block index) of open voxel j with par entry pj (k_descent_init with cr)
__device__ __forceinline__ uint32_t basin_root(uint32_t pj, uint32_t j) { return (pj & kDescRes) ? j : pj; }

// masked blocks (k_plateau.hip): the plateau voxels are walls until the plateau fill, and an
// open voxel whose descent ends in the plateau has no catchment here (its key stays INF; the
// frontier relaxation after the fill and the checked repair reach it)
__device__ __forceinline__ bool in_plat(const uint64_t* pb, const BlockDesc& B, int wpr, uint32_t j) {
    if (!pb) return false;
    const uint32_t row = j / (uint32_t)B.X, x = j - row * (uint32_t)B.X;
    return (gbl(pb)[(int64_t)row * wpr + (x >> 6)] >> (x & 63)) & 1ull;
}

// neighbour class from the open / plateau-wall bitmaps: 0 final, 1 open, 2 wall or outside
__device__ __forceinline__ int nclass(uint64_t ow, uint64_t pw, int bit) {
    if ((pw >> bit) & 1ull) return 2;
    return ((ow >> bit) & 1ull) ? 1 : 0;
}

// min of v over the run of equal (a, b) in lane order that contains this lane; `end` = the lane
// is the last of its run (its result covers the whole run)
__device__ __forceinline__ uint32_t run_min(uint32_t a, uint32_t b, uint32_t v, int lane, bool& end) {
    const uint32_t pa = (uint32_t)__shfl_up((int)a, 1), pb = (uint32_t)__shfl_up((int)b, 1);
    const bool start = lane == 0 || pa != a || pb != b;
    const uint64_t sm = __ballot(start) & ((2ull << lane) - 1ull);  // lane 63: all bits
    const int rs = 63 - __builtin_clzll(sm);
_Pragma("unroll")
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)v, off);
        if (lane - off >= rs) v = min(v, o);
    }
    const uint32_t na = (uint32_t)__shfl_down((int)a, 1), nb = (uint32_t)__shfl_down((int)b, 1);
    end = lane == 63 || na != a || nb != b;
    return v;
}

// The neighbourhood of one word of a row: the bitmap words around it (wave-uniform loads) and,
// per lane, the class and block index of each neighbour (order -x, +x, -y, +y, -z, +z).
template <int ND>
struct WordNbrs {
    static constexpr int K = 2 * ND;
    int cls[K];
    uint32_t idx[K];
    __device__ WordNbrs(const BlockDesc& B, const uint64_t* open, const uint64_t* plat, int64_t w, int wpr, int z,
                        int y, int xw, int lane, uint64_t ow, uint64_t pw) {
        const int x = xw * 64 + lane;
        const uint32_t i = (uint32_t)(((int64_t)z * B.Y + y) * B.X + x);
        const uint64_t* ob = open + B.fbase;
        const uint64_t* pb = plat ? plat + B.fbase : nullptr;
        // -x / +x
        {
            const bool in = x > 0;
            uint64_t o = ow, p = pw;
            int bit = lane - 1;
            if (lane == 0) {
                o = xw > 0 ? gbl(ob)[w - 1] : 0ull;
                p = (xw > 0 && pb) ? gbl(pb)[w - 1] : 0ull;
                bit = 63;
            }
            cls[0] = in ? nclass(o, p, bit) : 2;
            idx[0] = i - 1u;
        }
        {
            const bool in = x + 1 < B.X;
            uint64_t o = ow, p = pw;
            int bit = lane + 1;
            if (lane == 63) {
                o = xw + 1 < wpr ? gbl(ob)[w + 1] : 0ull;
                p = (xw + 1 < wpr && pb) ? gbl(pb)[w + 1] : 0ull;
                bit = 0;
            }
            cls[1] = in ? nclass(o, p, bit) : 2;
            idx[1] = i + 1u;
        }
        // -y / +y (, -z / +z): whole words, the same for every lane
        const int64_t ws[2] = {(int64_t)wpr, (int64_t)B.Y * wpr};
        const bool has[4] = {y > 0, y + 1 < B.Y, z > 0, z + 1 < B.Z};
        const uint32_t vs[2] = {(uint32_t)B.X, (uint32_t)B.Y * (uint32_t)B.X};
_Pragma("unroll")
        for (int k = 2; k < K; ++k) {
            const int ax = (k - 2) >> 1, dir = (k & 1) ? 1 : -1;
            const bool in = has[k - 2];
            const int64_t wn = w + dir * ws[ax];
            const uint64_t o = in ? gbl(ob)[wn] : 0ull;
            const uint64_t p = (in && pb) ? gbl(pb)[wn] : 0ull;
            cls[k] = in ? nclass(o, p, lane) : 2;
            idx[k] = dir > 0 ? i + vs[ax] : i - vs[ax];
        }
    }
};

// Phase 2a: C(root) from final neighbours (atomicMin), catchment pairs into the edge list.  The
// pairs of a workgroup collect in LDS and go out with one atomicAdd on the list length per
// workgroup (one per wave and direction serialised on that one address: 59 ms per batch).
constexpr int kEdgeStage = 2048;
template <int ND>
__global__ void __launch_bounds__(256) k_basin_edges(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     const float* __restrict__ h, const uint32_t* __restrict__ par,
                                                     const uint64_t* __restrict__ open, const uint64_t* __restrict__ plat,
                                                     uint32_t* __restrict__ cr, uint4* __restrict__ edges,
                                                     uint32_t* __restrict__ ecnt, uint32_t ecap) {
    __shared__ uint4 sbuf[kEdgeStage];
    __shared__ uint32_t scnt, sbase;
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    if (threadIdx.x == 0) scnt = 0u;
    __syncthreads();
    // word columns as k_flood_verify: a unit is U vertically adjacent words of one 64-voxel column;
    // its U + 2 rows of par / h / bitmap words are loaded once (all in flight) and serve as centre,
    // upper and lower rows; x-neighbours are lane shuffles, lane 0 / 63 load the voxel beyond
    constexpr int U = 4, R = U + 2, K = 2 * ND;
    const gptr_t<float> hb = gbl(h + B.base);
    const gptr_t<uint32_t> pr = gbl(par + B.base);
    const uint64_t* ob = open + B.fbase;
    const uint64_t* pbb = plat ? plat + B.fbase : nullptr;
    const int64_t YX = (int64_t)B.Y * B.X;
    const int wpr = (B.X + 63) >> 6;
    const int ngy = (B.Y + U - 1) / U;
    const int64_t nunits = (int64_t)B.Z * wpr * ngy;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nunits + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t ubeg = wid * per, uend = min(nunits, ubeg + per);
    for (int64_t un = ubeg; un < uend; ++un) {
        const int gy = (int)(un % ngy);
        const int64_t strip = un / ngy;
        const int xw = (int)(strip % wpr), z = (int)(strip / wpr);
        const int y0 = gy * U;
        const int64_t wrow0 = (int64_t)z * B.Y * wpr + xw;  // word of row y = 0 of the column
        uint64_t ow[R], pw[R];
        bool any = false;
_Pragma("unroll")
        for (int q = 0; q < R; ++q) {
            const int yy = y0 - 1 + q;
            const bool in = yy >= 0 && yy < B.Y;
            ow[q] = in ? gbl(ob)[wrow0 + (int64_t)yy * wpr] : 0ull;
            pw[q] = (in && pbb) ? gbl(pbb)[wrow0 + (int64_t)yy * wpr] : 0ull;
            if (q >= 1 && q <= U) any |= ow[q] != 0ull;
        }
        if (!any) continue;
        const int x = xw * 64 + lane;
        const int xc = min(x, B.X - 1);
        const int xe = lane == 0 ? max(xc - 1, 0) : min(xc + 1, B.X - 1);
        const int64_t zb = (int64_t)z * YX;
        uint32_t pv[R];
        float hv[R];
_Pragma("unroll")
        for (int q = 0; q < R; ++q) {
            const int yy = min(max(y0 - 1 + q, 0), B.Y - 1);
            pv[q] = pr[zb + (int64_t)yy * B.X + xc];
            hv[q] = hb[zb + (int64_t)yy * B.X + xc];
        }
        uint32_t pe[U], pzm[U], pzp[U];
        float he[U], hzm[U], hzp[U];
        uint64_t owe[U], pwe[U], owzm[U], pwzm[U], owzp[U], pwzp[U];
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            const int yy = min(y0 + u, B.Y - 1);
            const int64_t ic = zb + (int64_t)yy * B.X + xc;
            pe[u] = pr[zb + (int64_t)yy * B.X + xe];
            he[u] = hb[zb + (int64_t)yy * B.X + xe];
            // the bitmap word beyond the lane's word edge (lane 0: left, the others: right)
            const int xwe = lane == 0 ? xw - 1 : xw + 1;
            const bool ine = xwe >= 0 && xwe < wpr;
            const int64_t we = (int64_t)z * B.Y * wpr + (int64_t)yy * wpr + (ine ? xwe : xw);
            owe[u] = ine ? gbl(ob)[we] : 0ull;
            pwe[u] = (ine && pbb) ? gbl(pbb)[we] : 0ull;
            if (ND == 3) {
                const int64_t wz = wrow0 + (int64_t)yy * wpr;
                const int64_t sw = (int64_t)B.Y * wpr;
                pzm[u] = pr[z > 0 ? ic - YX : ic];
                pzp[u] = pr[z + 1 < B.Z ? ic + YX : ic];
                hzm[u] = hb[z > 0 ? ic - YX : ic];
                hzp[u] = hb[z + 1 < B.Z ? ic + YX : ic];
                owzm[u] = z > 0 ? gbl(ob)[wz - sw] : 0ull;
                owzp[u] = z + 1 < B.Z ? gbl(ob)[wz + sw] : 0ull;
                pwzm[u] = (z > 0 && pbb) ? gbl(pbb)[wz - sw] : 0ull;
                pwzp[u] = (z + 1 < B.Z && pbb) ? gbl(pbb)[wz + sw] : 0ull;
            }
        }
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            const int y = y0 + u;
            const bool me = y < B.Y && x < B.X && ((ow[u + 1] >> lane) & 1ull);
            const uint32_t i = (uint32_t)(zb + (int64_t)y * B.X + x);
            // x-neighbours from the neighbouring lanes (every lane shuffles)
            const uint32_t pxm = (uint32_t)__shfl_up((int)pv[u + 1], 1), pxp = (uint32_t)__shfl_down((int)pv[u + 1], 1);
            const float hxm = __shfl_up(hv[u + 1], 1), hxp = __shfl_down(hv[u + 1], 1);
            uint32_t A = me ? basin_root(pv[u + 1], i) : 0xFFFFFFFFu;
            const bool live = me && !in_plat(pbb, B, wpr, A);
            if (!live) A = 0xFFFFFFFFu;
            const uint32_t hq = ordf(hv[u + 1]);
            int cls[K];
            uint32_t np[K], nj[K];
            float nh[K];
            cls[0] = x > 0 ? (lane > 0 ? nclass(ow[u + 1], pw[u + 1], lane - 1) : nclass(owe[u], pwe[u], 63)) : 2;
            np[0] = lane > 0 ? pxm : pe[u];
            nh[0] = lane > 0 ? hxm : he[u];
            nj[0] = i - 1u;
            cls[1] = x + 1 < B.X ? (lane < 63 ? nclass(ow[u + 1], pw[u + 1], lane + 1) : nclass(owe[u], pwe[u], 0)) : 2;
            np[1] = lane < 63 ? pxp : pe[u];
            nh[1] = lane < 63 ? hxp : he[u];
            nj[1] = i + 1u;
            cls[2] = y > 0 ? nclass(ow[u], pw[u], lane) : 2;
            np[2] = pv[u];
            nh[2] = hv[u];
            nj[2] = i - (uint32_t)B.X;
            cls[3] = y + 1 < B.Y ? nclass(ow[u + 2], pw[u + 2], lane) : 2;
            np[3] = pv[u + 2];
            nh[3] = hv[u + 2];
            nj[3] = i + (uint32_t)B.X;
            if (ND == 3) {
                cls[4] = z > 0 ? nclass(owzm[u], pwzm[u], lane) : 2;
                np[4] = pzm[u];
                nh[4] = hzm[u];
                nj[4] = i - (uint32_t)YX;
                cls[5] = z + 1 < B.Z ? nclass(owzp[u], pwzp[u], lane) : 2;
                np[5] = pzp[u];
                nh[5] = hzp[u];
                nj[5] = i + (uint32_t)YX;
            }
            uint32_t mres = 0xFFFFFFFFu;
            uint32_t eb[K], ew[K];
_Pragma("unroll")
            for (int k = 0; k < K; ++k) {
                eb[k] = 0xFFFFFFFFu;
                ew[k] = 0xFFFFFFFFu;
                const int c = live ? cls[k] : 2;
                if (c == 2) continue;
                const uint32_t w2 = max(hq, ordf(nh[k]));
                if (c == 0) {
                    mres = min(mres, w2);
                } else {
                    const uint32_t Bj = basin_root(np[k], nj[k]);
                    if (Bj != A && !in_plat(pbb, B, wpr, Bj)) {
                        eb[k] = Bj;
                        ew[k] = w2;
                    }
                }
            }
            bool end;
            const uint32_t m = run_min(A, 0u, mres, lane, end);
            if (end && live && m != 0xFFFFFFFFu) atomic_min_if(&cr[B.base + A], m);
_Pragma("unroll")
            for (int k = 0; k < K; ++k) {
                const uint32_t wm = run_min(A, eb[k], ew[k], lane, end);
                const bool app = end && eb[k] != 0xFFFFFFFFu;
                const uint64_t am = __ballot(app);
                if (!am) continue;
                const uint32_t n = (uint32_t)__popcll(am);
                const uint32_t rank = (uint32_t)__popcll(am & ((1ull << lane) - 1ull));
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&scnt, n);  // LDS
                base = (uint32_t)__shfl((int)base, 0);
                const bool to_lds = base + n <= (uint32_t)kEdgeStage;
                const uint4 ev = make_uint4((uint32_t)(B.base + A), (uint32_t)(B.base + eb[k]), wm, 0u);
                if (to_lds) {
                    if (app) sbuf[base + rank] = ev;
                } else {
                    // stage full: straight out; the reserved stage slots get a self-pair (no effect)
                    if (app && base + rank < (uint32_t)kEdgeStage) sbuf[base + rank] = make_uint4(0u, 0u, 0xFFFFFFFFu, 0u);
                    uint32_t gb = 0;
                    if (lane == 0) gb = atomicAdd(ecnt, n);
                    gb = (uint32_t)__shfl((int)gb, 0);
                    if (app && gb + rank < ecap) edges[gb + rank] = ev;
                }
            }
        }
    }
    __syncthreads();
    const uint32_t ns = min(scnt, (uint32_t)kEdgeStage);
    if (threadIdx.x == 0) sbase = ns ? atomicAdd(ecnt, ns) : 0u;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < ns; t += blockDim.x)
        if (sbase + t < ecap) edges[sbase + t] = sbuf[t];
}

// Phase 2b: one Bellman-Ford sweep over the catchment pairs; flags[it] = a root's C changed.
// Iteration it returns at once when iteration it - 1 changed nothing (converged).
__global__ void __launch_bounds__(256) k_basin_relax(const uint4* __restrict__ edges, const uint32_t* __restrict__ ecnt,
                                                     uint32_t ecap, uint32_t* __restrict__ cr, uint32_t* __restrict__ flags,
                                                     int it) {
    if (it > 0 && flags[it - 1] == 0u) return;
    const uint32_t n = min(*ecnt, ecap);
    bool ch = false;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        const uint4 ed = edges[e];
        const uint32_t c = max(ed.z, cr[ed.y]);
        if (c < cr[ed.x]) {
            atomicMin(&cr[ed.x], c);
            ch = true;
        }
    }
    if (__ballot(ch) && (threadIdx.x & 63) == 0) atomicOr(&flags[it], 1u);
}

// Phase 3a: C of every open voxel, key (C, 0, 0) (INF for a catchment without a pass to a seed,
// or whose root is a masked-plateau voxel).  Contiguous word ranges per wave, U words in flight
// (the root's C is a dependent gather).
__global__ void __launch_bounds__(256) k_basin_c(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                 const float* __restrict__ h, const uint32_t* __restrict__ par,
                                                 const uint64_t* __restrict__ open, const uint64_t* __restrict__ plat,
                                                 const uint32_t* __restrict__ cr, uint64_t* __restrict__ key) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    constexpr int U = 4;
    const int wpr = (B.X + 63) >> 6;
    const int64_t nwords = (int64_t)B.Z * B.Y * wpr;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nwords + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t wbeg = wid * per, wend = min(nwords, wbeg + per);
    const gptr_t<uint32_t> pr = gbl(par + B.base);
    const gptr_t<float> hb = gbl(h + B.base);
    const gptr_t<uint32_t> crb = gbl(cr + B.base);
    const uint64_t* pbb = plat ? plat + B.fbase : nullptr;
    for (int64_t w0 = wbeg; w0 < wend; w0 += U) {
        uint64_t ow[U];
        bool any = false;
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            ow[u] = w0 + u < wend ? gbl(open)[B.fbase + w0 + u] : 0ull;
            any |= ow[u] != 0ull;
        }
        if (!any) continue;
        uint32_t gi[U], pv[U];
        bool me[U];
        float hv[U];
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            const int64_t row = (w0 + u) / wpr;
            const int x = (int)(w0 + u - row * wpr) * 64 + lane;
            me[u] = ((ow[u] >> lane) & 1ull) && x < B.X;
            gi[u] = me[u] ? (uint32_t)(row * B.X + x) : 0u;
            pv[u] = pr[gi[u]];
            hv[u] = hb[gi[u]];
        }
        uint32_t rt[U], cv[U];
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            rt[u] = basin_root(pv[u], gi[u]);
            cv[u] = crb[rt[u]];
        }
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            if (!me[u]) continue;
            const bool dead = cv[u] == 0xFFFFFFFFu || in_plat(pbb, B, wpr, rt[u]);
            key[B.base + gi[u]] = dead ? kPackInf : ((uint64_t)max(ordf(hv[u]), cv[u]) << 32);
        }
    }
}

// Phase 3b: the lake voxels (open, reached, h(q) <= min_p C(p)) -> the lake bitmap (the open set of
// the lake relaxation), `chg` = every other voxel (its first changed set).  A stencil over the
// keys of 3a (C of every voxel: h of a final one, INF at walls): word columns as k_flood_verify.
// The lake keys are reset to INF afterwards (k_basin_lake_reset), not here: the neighbours still
// read them.  nlake[0] += lake voxels.
template <int ND>
__global__ void __launch_bounds__(256) k_basin_keys(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    const float* __restrict__ h, const uint64_t* __restrict__ open,
                                                    const uint64_t* __restrict__ key, uint64_t* __restrict__ lake,
                                                    uint64_t* __restrict__ chg, uint32_t* __restrict__ nlake) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    constexpr int U = 4, R = U + 2;
    const gptr_t<uint64_t> k = gbl(key + B.base);
    const gptr_t<float> hb = gbl(h + B.base);
    const int64_t YX = (int64_t)B.Y * B.X;
    const int wpr = (B.X + 63) >> 6;
    const int ngy = (B.Y + U - 1) / U;
    const int64_t nunits = (int64_t)B.Z * wpr * ngy;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nunits + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t ubeg = wid * per, uend = min(nunits, ubeg + per);
    uint32_t cnt = 0;
    for (int64_t un = ubeg; un < uend; ++un) {
        const int gy = (int)(un % ngy);
        const int64_t strip = un / ngy;
        const int xw = (int)(strip % wpr), z = (int)(strip / wpr);
        const int y0 = gy * U;
        const uint64_t vm = (B.X - xw * 64 >= 64) ? ~0ull : ((1ull << (B.X - xw * 64)) - 1ull);
        uint64_t ow[U], lw[U];
        bool any = false;
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            ow[u] = y0 + u < B.Y ? gbl(open)[B.fbase + ((int64_t)z * B.Y + y0 + u) * wpr + xw] : 0ull;
            any |= ow[u] != 0ull;
            lw[u] = 0ull;
        }
        if (any) {
            const int x = xw * 64 + lane;
            const int xc = min(x, B.X - 1);
            const int xe = lane == 0 ? max(xc - 1, 0) : min(xc + 1, B.X - 1);
            const int64_t zb = (int64_t)z * YX;
            uint64_t rk[R];
_Pragma("unroll")
            for (int q = 0; q < R; ++q) {
                const int yy = min(max(y0 - 1 + q, 0), B.Y - 1);
                rk[q] = k[zb + (int64_t)yy * B.X + xc];
            }
            uint64_t ke[U], kzm[U], kzp[U];
            float hv[U];
_Pragma("unroll")
            for (int u = 0; u < U; ++u) {
                const int yy = min(y0 + u, B.Y - 1);
                const int64_t ic = zb + (int64_t)yy * B.X + xc;
                ke[u] = k[zb + (int64_t)yy * B.X + xe];
                hv[u] = hb[ic];
                if (ND == 3) {
                    kzm[u] = k[z > 0 ? ic - YX : ic];
                    kzp[u] = k[z + 1 < B.Z ? ic + YX : ic];
                }
            }
_Pragma("unroll")
            for (int u = 0; u < U; ++u) {
                const int y = y0 + u;
                const bool valid = y < B.Y && x < B.X;
                const uint64_t o = valid ? rk[u + 1] : kPackInf;
                uint64_t l = shfl_up_u64(o, 1), r = shfl_down_u64(o, 1);
                const uint64_t ker = shfl_u64(ke[u], 63);
                if (lane == 0) l = (x > 0) ? ke[u] : kPackInf;
                if (lane == 63) r = ker;
                if (x + 1 >= B.X) r = kPackInf;
                uint64_t m = min(l, r);
                if (y > 0) m = min(m, rk[u]);
                if (y + 1 < B.Y) m = min(m, rk[u + 2]);
                if (ND == 3) {
                    if (z > 0) m = min(m, kzm[u]);
                    if (z + 1 < B.Z) m = min(m, kzp[u]);
                }
                const bool isl = valid && ((ow[u] >> lane) & 1ull) && o != kPackInf &&
                                 ordf(hv[u]) <= (uint32_t)(m >> 32);
                lw[u] = __ballot(isl);
            }
        }
        if (lane == 0) {
_Pragma("unroll")
            for (int u = 0; u < U; ++u) {
                if (y0 + u >= B.Y) continue;
                const int64_t w = ((int64_t)z * B.Y + y0 + u) * wpr + xw;
                lake[B.fbase + w] = lw[u];
                chg[B.fbase + w] = ~lw[u] & vm;
                cnt += (uint32_t)__popcll(lw[u]);
            }
        }
    }
    cnt = wg_reduce_u32(cnt, OpAdd());
    if (threadIdx.x == 0 && cnt) atomicAdd(nlake, cnt);
}

// Phase 3c: the lake voxels' keys -> INF (the lake relaxation's starting point: upper bounds)
__global__ void __launch_bounds__(256) k_basin_lake_reset(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                          const uint64_t* __restrict__ lake, uint64_t* __restrict__ key) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int wpr = (B.X + 63) >> 6;
    const int64_t nw = (int64_t)B.Z * B.Y * wpr;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t bits = lake[B.fbase + w];
        if (!bits) continue;
        const int64_t row = w / wpr;
        const int xw = (int)(w - row * wpr);
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            key[B.base + row * B.X + xw * 64 + b] = kPackInf;
        }
    }
}

// Phase 4a: parents by argmin (C, d) and their chains inside a tile (tile + 1-voxel halo of keys
// in LDS, pointer jumping as k_descent_tile).  par[q] of an open voxel := kDescRes | label when
// its chain ends at a final voxel of the tile or its halo (0: unreached), else the block index
// of the first open halo voxel on it (k_basin_hop follows those).
template <int ND>
__global__ void __launch_bounds__(512) k_basin_tile(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    const uint64_t* __restrict__ key, const uint64_t* __restrict__ open,
                                                    const uint64_t* __restrict__ plat, uint32_t* __restrict__ par) {
    constexpr int NT = 512;
    constexpr int TZ = ND == 3 ? 16 : 1, TY = ND == 3 ? 16 : 64, TX = ND == 3 ? 16 : 64, HZ = ND == 3 ? 18 : 1;
    constexpr int HY = TY + 2, HX = TX + 2, HN = HZ * HY * HX, TN = TZ * TY * TX;
    constexpr int ZOFF = ND == 3 ? 1 : 0;
    constexpr int PER = TN / NT;
    static_assert(TN % NT == 0 && TN + HN < 32768, "");
    __shared__ uint64_t sk[HN];  // keys (kPackInf outside the block and at walls)
    __shared__ uint8_t sc[HN];   // class: 0 final, 1 open, 2 wall / outside
    __shared__ int16_t sp[TN];   // pointer: < TN tile voxel, >= TN halo voxel (TN + halo index)
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int ntx = (B.X + TX - 1) / TX, nty = (B.Y + TY - 1) / TY, ntz = (B.Z + TZ - 1) / TZ;
    const int t = blockIdx.x;
    if (t >= ntx * nty * ntz) return;
    const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    const int64_t YX = (int64_t)B.Y * B.X;
    const int wpr = (B.X + 63) >> 6;
    const uint64_t* ob = open + B.fbase;
    const uint64_t* pb = plat ? plat + B.fbase : nullptr;
    // any open voxel in the tile?  (rows of the tile: TZ * TY words, TX bits of each)
    {
        bool any = false;
        for (int r = threadIdx.x; r < TZ * TY; r += NT) {
            const int lz = r / TY, ly = r % TY;
            const int gz = z0 + lz, gy = y0 + ly;
            if (gz < B.Z && gy < B.Y) {
                const uint64_t wv = gbl(ob)[((int64_t)gz * B.Y + gy) * wpr + (x0 >> 6)];
                const uint64_t m = TX == 64 ? ~0ull : (((1ull << TX) - 1ull) << (x0 & 63));
                any |= (wv & m) != 0ull;
            }
        }
        if (!__syncthreads_or(any)) return;
    }
    const gptr_t<uint64_t> kb = gbl(key + B.base);
    {
        constexpr int NH = (HN + NT - 1) / NT;
        uint64_t kv[NH];
        uint64_t ov[NH], pv[NH];
_Pragma("unroll")
        for (int k = 0; k < NH; ++k) {
            const int c = min((int)threadIdx.x + k * NT, HN - 1);
            const int hx = c % HX, hy = (c / HX) % HY, hz = c / (HX * HY);
            const int gz = z0 + hz - ZOFF, gy = y0 + hy - 1, gx = x0 + hx - 1;
            const int cz = min(max(gz, 0), B.Z - 1), cy = min(max(gy, 0), B.Y - 1), cx = min(max(gx, 0), B.X - 1);
            kv[k] = kb[cz * YX + (int64_t)cy * B.X + cx];
            const int64_t wi = ((int64_t)cz * B.Y + cy) * wpr + (cx >> 6);
            ov[k] = gbl(ob)[wi];
            pv[k] = pb ? gbl(pb)[wi] : 0ull;
        }
_Pragma("unroll")
        for (int k = 0; k < NH; ++k) {
            const int c = (int)threadIdx.x + k * NT;
            if (c < HN) {
                const int hx = c % HX, hy = (c / HX) % HY, hz = c / (HX * HY);
                const int gz = z0 + hz - ZOFF, gy = y0 + hy - 1, gx = x0 + hx - 1;
                const bool out = gz < 0 || gz >= B.Z || gy < 0 || gy >= B.Y || gx < 0 || gx >= B.X;
                const int cl = out ? 2 : nclass(ov[k], pv[k], gx & 63);
                sc[c] = (uint8_t)cl;
                sk[c] = cl == 2 ? kPackInf : kv[k];
            }
        }
    }
    __syncthreads();
    // parents of the open tile voxels: the first argmin (C, d) neighbour (none: unreached)
_Pragma("unroll")
    for (int k = 0; k < PER; ++k) {
        const int c = threadIdx.x + k * NT;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int hc = ((lz + ZOFF) * HY + ly + 1) * HX + lx + 1;
        int p = c;
        if (sc[hc] == 1 && sk[hc] != kPackInf) {  // (an INF key: unreached here, left to the repair)
            uint64_t best = kPackInf >> kLabelBits;
            int bh = -1;
            auto cand = [&](int o) {
                const uint64_t v = sk[hc + o] >> kLabelBits;
                if (v < best) {
                    best = v;
                    bh = hc + o;
                }
            };
            cand(-1);
            cand(1);
            cand(-HX);
            cand(HX);
            if (ND == 3) {
                cand(-HX * HY);
                cand(HX * HY);
            }
            if (bh >= 0) {
                const int hx = bh % HX, hy = (bh / HX) % HY, hz = bh / (HX * HY);
                const bool inside = hx >= 1 && hx <= TX && hy >= 1 && hy <= TY && (ND == 2 || (hz >= 1 && hz <= TZ));
                p = inside ? ((hz - ZOFF) * TY + (hy - 1)) * TX + (hx - 1) : TN + bh;
            }
        }
        sp[c] = (int16_t)p;
    }
    __syncthreads();
    for (int it = 0; it < 16; ++it) {
        bool moved = false;
_Pragma("unroll")
        for (int k = 0; k < PER; ++k) {
            const int c = threadIdx.x + k * NT;
            const int p = sp[c];
            if (p < TN) {
                const int pp = sp[p];
                if (pp != p) {
                    sp[c] = (int16_t)pp;
                    moved = true;
                }
            }
        }
        if (!__syncthreads_or(moved)) break;
    }
_Pragma("unroll")
    for (int k = 0; k < PER; ++k) {
        const int c = threadIdx.x + k * NT;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int hc = ((lz + ZOFF) * HY + ly + 1) * HX + lx + 1;
        if (sc[hc] != 1) continue;  // final, wall or outside the block
        const int gz = z0 + lz, gy = y0 + ly, gx = x0 + lx;
        const int p = sp[c];
        int hr;  // halo-coordinate index of the chain's end in this tile
        if (p < TN) {
            const int rx = p % TX, ry = (p / TX) % TY, rz = p / (TX * TY);
            hr = ((rz + ZOFF) * HY + ry + 1) * HX + rx + 1;
        } else {
            hr = p - TN;
        }
        uint32_t e;
        if (sc[hr] == 0) {
            e = kDescRes | (uint32_t)(sk[hr] & kLabelMask);
        } else if (p >= TN && sc[hr] == 1) {
            const int ex = x0 + hr % HX - 1, ey = y0 + (hr / HX) % HY - 1, ez = z0 + hr / (HX * HY) - ZOFF;
            e = (uint32_t)(ez * YX + (int64_t)ey * B.X + ex);
        } else {
            e = kDescRes;  // unreached
        }
        par[B.base + gz * YX + (int64_t)gy * B.X + gx] = e;
    }
}

// Phase 4b: follow the chains across tiles (one hop per tile crossed) and write the labels.
__global__ void __launch_bounds__(256) k_basin_hop(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                   const uint32_t* __restrict__ par, const uint64_t* __restrict__ open,
                                                   uint64_t* __restrict__ key) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    constexpr int U = 4;
    const int wpr = (B.X + 63) >> 6;
    const int64_t nwords = (int64_t)B.Z * B.Y * wpr;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nwords + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t wbeg = wid * per, wend = min(nwords, wbeg + per);
    const gptr_t<uint32_t> pr = gbl(par + B.base);
    for (int64_t w0 = wbeg; w0 < wend; w0 += U) {
        uint64_t ow[U];
        bool any = false;
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            ow[u] = w0 + u < wend ? gbl(open)[B.fbase + w0 + u] : 0ull;
            any |= ow[u] != 0ull;
        }
        if (!any) continue;
        int64_t gi[U];
        bool me[U];
        uint32_t e[U];
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            const int64_t row = (w0 + u) / wpr;
            const int x = (int)(w0 + u - row * wpr) * 64 + lane;
            me[u] = ((ow[u] >> lane) & 1ull) && x < B.X;
            gi[u] = me[u] ? row * B.X + x : 0;
            e[u] = me[u] ? pr[gi[u]] : kDescRes;
        }
        for (int hop = 0; hop < 1 << 16; ++hop) {
            bool more = false;
_Pragma("unroll")
            for (int u = 0; u < U; ++u) more |= !(e[u] & kDescRes);
            if (!more) break;
_Pragma("unroll")
            for (int u = 0; u < U; ++u)
                if (!(e[u] & kDescRes)) e[u] = pr[e[u]];
        }
_Pragma("unroll")
        for (int u = 0; u < U; ++u) {
            const uint32_t l = e[u] & ~kDescRes;
            if (me[u] && l) {
                uint64_t* kp = key + B.base + gi[u];
                const uint64_t k0 = *kp;
                if (k0 != kPackInf) *kp = (k0 & ~kLabelMask) | (uint64_t)l;
            }
        }
    }
}

template __global__ void k_basin_edges<2>(const BlockDesc*, const BlockStat*, const float*, const uint32_t*,
                                          const uint64_t*, const uint64_t*, uint32_t*, uint4*, uint32_t*, uint32_t);
template __global__ void k_basin_edges<3>(const BlockDesc*, const BlockStat*, const float*, const uint32_t*,
                                          const uint64_t*, const uint64_t*, uint32_t*, uint4*, uint32_t*, uint32_t);
template __global__ void k_basin_keys<2>(const BlockDesc*, const BlockStat*, const float*, const uint64_t*,
                                         const uint64_t*, uint64_t*, uint64_t*, uint32_t*);
template __global__ void k_basin_keys<3>(const BlockDesc*, const BlockStat*, const float*, const uint64_t*,
                                         const uint64_t*, uint64_t*, uint64_t*, uint32_t*);
template __global__ void k_basin_tile<2>(const BlockDesc*, const BlockStat*, const uint64_t*, const uint64_t*,
                                         const uint64_t*, uint32_t*);
template __global__ void k_basin_tile<3>(const BlockDesc*, const BlockStat*, const uint64_t*, const uint64_t*,
                                         const uint64_t*, uint32_t*);

}  // namespace ctws
