// ctws_oracle.cpp — CPU restatement of cluster_tools' blockwise DT watershed.
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the CPU baseline
// ("port") of bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it.  The product path (cluster_tools_amd, libctws.so)
// never links or calls it.
//
// What it restates (reference = k-dominik/cluster_tools; paths relative to it):
//   _ws_block                 cluster_tools/watershed/watershed.py:285-341
//   _read_data / normalize    watershed.py:267-282, utils/volume_utils.py:113-120
//   _apply_dt                 watershed.py:139-160
//   _make_hmap                watershed.py:163-169
//   _make_seeds               watershed.py:179-207
//   _apply_watershed          watershed.py:211-249
//   vu.watershed / size filt. utils/volume_utils.py:123-139
//   _ws_pass2 (+with_seeds)   watershed/two_pass_watershed.py:122-255
// and the vigra algorithms those lines call.  vigra is a third-party dependency that
// is NOT present under /root/reference (environment.yml:12, unpinned; vigra 1.11-era
// semantics), so its published algorithms are restated here:
//   distanceTransform        -> separableMultiDistSquared + distParabola (Felzenszwalb-
//                               Huttenlocher lower envelope), float32 storage, sqrtf
//   gaussianSmoothing        -> Kernel1D::initGaussian (radius int(3*sigma+0.5)),
//                               normalize(1.0), convolveLine with BORDER_TREATMENT_REFLECT,
//                               double accumulation, ascending taps, float32 between axes
//   localMaxima[3D]          -> extendedLocalMinMax (plateaus, allowAtBorder, thresh -FLT_MAX)
//   labelMultiArrayWithBackground / labelVolumeWithBackground
//                            -> union-find, labels by first occurrence in vigra scan order
//   watershedsNew            -> seededWatersheds: std::priority_queue min-heap on the
//                               priority only, label-on-push, priority max(h, cost)
//   relabelConsecutive       -> first appearance in scan order, keep_zeros, start 1
// vigra scan order (Appendix A.0 of SURVEY.md): for plain numpy arrays vigra dim k is numpy
// axis k and dim 0 is iterated fastest, i.e. the F-order linear index.
//
// Parity status: vigra/nifty cannot be imported or built here, so these semantics are
// pinned only by cross-checks against scipy / scikit-image (tests/test_oracle_crosscheck.py)
// and by the reference's structural invariants (test/watershed/test_watershed.py:53-70).
// The watershed tie order follows libstdc++'s std::priority_queue, which is what vigra's
// PriorityQueue wraps.

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <queue>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../include/ctws.h"

namespace {

// ---------------------------------------------------------------------------------------
// N-d (N = 2 or 3) views in numpy order.  vigra dim k == numpy axis k.
// ---------------------------------------------------------------------------------------
struct Dims {
    int nd = 3;
    int64_t n[3] = {1, 1, 1};
    int64_t st[3] = {0, 0, 0};  // C-order strides in elements
    int64_t size = 1;
};

Dims make_dims(int nd, const int64_t* shape) {
    Dims d;
    d.nd = nd;
    for (int k = 0; k < nd; ++k) d.n[k] = shape[k];
    int64_t s = 1;
    for (int k = nd - 1; k >= 0; --k) {
        d.st[k] = s;
        s *= d.n[k];
    }
    d.size = s;
    return d;
}

// visit every element in vigra scan order (dim 0 fastest)
template <class F>
void scan_order(const Dims& d, F f) {
    if (d.nd == 2) {
        for (int64_t i1 = 0; i1 < d.n[1]; ++i1)
            for (int64_t i0 = 0; i0 < d.n[0]; ++i0) f(i0 * d.st[0] + i1 * d.st[1]);
    } else {
        for (int64_t i2 = 0; i2 < d.n[2]; ++i2)
            for (int64_t i1 = 0; i1 < d.n[1]; ++i1)
                for (int64_t i0 = 0; i0 < d.n[0]; ++i0)
                    f(i0 * d.st[0] + i1 * d.st[1] + i2 * d.st[2]);
    }
}

inline void coords(const Dims& d, int64_t idx, int64_t* c) {
    for (int k = 0; k < d.nd; ++k) {
        c[k] = idx / d.st[k];
        idx -= c[k] * d.st[k];
    }
}

// Direct neighbourhood in vigra order (MakeDirectArrayNeighborhood<N-1>):
//   -e_{N-1}, ..., -e_0, +e_0, ..., +e_{N-1}.  The first N are the "back" neighbours.
struct Nbr {
    int dim;
    int sign;
};
std::vector<Nbr> direct_nbrs(int nd) {
    std::vector<Nbr> v;
    for (int k = nd - 1; k >= 0; --k) v.push_back({k, -1});
    for (int k = 0; k < nd; ++k) v.push_back({k, +1});
    return v;
}

// all neighbours with offsets in {-1,0,1}^nd \ 0 (8-nbhd in 2-D), as coordinate deltas
std::vector<std::array<int, 3>> indirect_deltas(int nd) {
    std::vector<std::array<int, 3>> v;
    if (nd == 2) {
        for (int a = -1; a <= 1; ++a)
            for (int b = -1; b <= 1; ++b)
                if (a || b) v.push_back({a, b, 0});
    } else {
        for (int a = -1; a <= 1; ++a)
            for (int b = -1; b <= 1; ++b)
                for (int c = -1; c <= 1; ++c)
                    if (a || b || c) v.push_back({a, b, c});
    }
    return v;
}

// ---------------------------------------------------------------------------------------
// Union-find with scan-order roots (vigra detail::UnionFindArray semantics: the root of a
// merged set is the smaller index; indices are handed out in scan order).
// ---------------------------------------------------------------------------------------
struct UF {
    std::vector<int64_t> p;
    explicit UF(int64_t n) : p(n) {
        for (int64_t i = 0; i < n; ++i) p[i] = i;
    }
    int64_t find(int64_t a) {
        int64_t r = a;
        while (p[r] != r) r = p[r];
        while (p[a] != r) {
            int64_t n = p[a];
            p[a] = r;
            a = n;
        }
        return r;
    }
    void unite(int64_t a, int64_t b) {
        a = find(a);
        b = find(b);
        if (a == b) return;
        if (a < b) p[b] = a;
        else p[a] = b;
    }
};

// ---------------------------------------------------------------------------------------
// labelMultiArrayWithBackground / labelVolumeWithBackground (vigra labelGraphWithBackground)
// CC of equal, non-background values under the direct neighbourhood; labels 1..k in order of
// each component's first voxel in scan order.  Returns k.
// ---------------------------------------------------------------------------------------
template <class T>
uint32_t label_with_background(const T* in, const Dims& d, T background, uint32_t* out) {
    // scan position of each element so that "smaller index" == "earlier in scan order"
    std::vector<int64_t> order;  // scan position -> linear idx
    order.reserve(d.size);
    scan_order(d, [&](int64_t i) { order.push_back(i); });
    std::vector<int64_t> pos(d.size);
    for (int64_t s = 0; s < d.size; ++s) pos[order[s]] = s;
    UF uf(d.size);
    auto nb = direct_nbrs(d.nd);
    int64_t c[3];
    for (int64_t s = 0; s < d.size; ++s) {
        int64_t i = order[s];
        if (in[i] == background) continue;
        coords(d, i, c);
        for (int q = 0; q < d.nd; ++q) {  // back neighbours
            const Nbr& e = nb[q];
            if (c[e.dim] == 0) continue;
            int64_t j = i - d.st[e.dim];
            if (in[j] == in[i]) uf.unite(pos[i], pos[j]);
        }
    }
    std::vector<uint32_t> lab(d.size, 0);
    uint32_t count = 0;
    for (int64_t s = 0; s < d.size; ++s) {
        int64_t i = order[s];
        if (in[i] == background) {
            out[i] = 0;
            continue;
        }
        int64_t r = uf.find(s);
        if (lab[r] == 0) lab[r] = ++count;
        out[i] = lab[r];
    }
    return count;
}

// ---------------------------------------------------------------------------------------
// vigra distanceTransform (background=True): separableMultiDistSquared + sqrt.
// fg != 0 voxels are "non-background" (distance 0).  The other voxels get the distance to
// the nearest fg voxel; with no fg at all every voxel is sqrt(ceil(dmax)).
// ---------------------------------------------------------------------------------------
template <class Tmp>
struct ParabolaEntry {
    double left, center, right;
    Tmp prevVal;
};

// detail::distParabola: lower envelope of parabolas sigma^2 (x - c)^2 + f(c)
template <class Tmp, class Dst>
void dist_parabola(const Tmp* line, int64_t w_, Dst* out, int64_t ostride, double sigma) {
    double w = (double)w_;
    if (w <= 0) return;
    double sigma2 = sigma * sigma;
    double sigma22 = 2.0 * sigma2;
    std::vector<ParabolaEntry<Tmp>> stack;
    stack.push_back({0.0, 0.0, w, line[0]});
    double current = 1.0;
    int64_t is = 1;
    for (; current < w; ++is, ++current) {
        double intersection;
        while (true) {
            ParabolaEntry<Tmp>& s = stack.back();
            double diff = current - s.center;
            intersection = current + (line[is] - s.prevVal - sigma2 * (diff * diff)) / (sigma22 * diff);
            if (intersection < s.left) {
                stack.pop_back();
                if (stack.empty()) {
                    intersection = 0.0;
                    break;
                }
                continue;
            } else if (intersection < s.right) {
                s.right = intersection;
            }
            break;
        }
        stack.push_back({intersection, current, w, line[is]});
    }
    size_t it = 0;
    int64_t o = 0;
    for (current = 0.0; current < w; ++current, ++o) {
        while (current >= stack[it].right) ++it;
        double diff = current - stack[it].center;
        out[o * ostride] = (Dst)(sigma2 * (diff * diff) + stack[it].prevVal);
    }
}

template <class T>
void dist_passes(T* arr, const Dims& d, const double* pitch) {
    std::vector<T> tmp;
    for (int k = 0; k < d.nd; ++k) {
        int64_t n = d.n[k], st = d.st[k];
        tmp.resize(n);
        // iterate over all lines along dim k
        for (int64_t base = 0; base < d.size; ++base) {
            int64_t c[3];
            coords(d, base, c);
            if (c[k] != 0) continue;
            for (int64_t i = 0; i < n; ++i) tmp[i] = arr[base + i * st];
            dist_parabola<T, T>(tmp.data(), n, arr + base, st, pitch[k]);
        }
    }
}

void distance_transform(const uint8_t* fg, const Dims& d, const double* pitch_in, float* out) {
    double pitch[3] = {1.0, 1.0, 1.0};
    if (pitch_in)
        for (int k = 0; k < d.nd; ++k) pitch[k] = pitch_in[k];
    double dmax = 0.0;
    bool real_pitch = false;
    for (int k = 0; k < d.nd; ++k) {
        if ((double)(int)pitch[k] != pitch[k]) real_pitch = true;
        dmax += (pitch[k] * d.n[k]) * (pitch[k] * d.n[k]);
    }
    if (dmax > (double)FLT_MAX || real_pitch) {
        std::vector<double> tmp(d.size);
        double maxDist = dmax;
        for (int64_t i = 0; i < d.size; ++i) tmp[i] = fg[i] ? 0.0 : maxDist;
        dist_passes<double>(tmp.data(), d, pitch);
        for (int64_t i = 0; i < d.size; ++i) out[i] = (float)tmp[i];
    } else {
        float maxDist = (float)std::ceil(dmax);
        for (int64_t i = 0; i < d.size; ++i) out[i] = fg[i] ? 0.0f : maxDist;
        dist_passes<float>(out, d, pitch);
    }
    for (int64_t i = 0; i < d.size; ++i) out[i] = std::sqrt(out[i]);
}

// ---------------------------------------------------------------------------------------
// vigra gaussianSmoothing
// ---------------------------------------------------------------------------------------
// Kernel1D<double>::initGaussian(sigma, 1.0, 0.0)
std::vector<double> gaussian_kernel(double sigma) {
    std::vector<double> k;
    if (sigma > 0.0) {
        double s = sigma;
        double sigma2 = -0.5 / s / s;
        double norm = 1.0 / (std::sqrt(2.0 * M_PI) * s);
        int radius = (int)(3.0 * sigma + 0.5);
        if (radius == 0) radius = 1;
        for (double x = -(double)radius; x <= (double)radius; ++x) {
            double x2 = x * x;
            k.push_back(norm * std::exp(x2 * sigma2));
        }
    } else {
        k.push_back(1.0);
    }
    double sum = 0.0;
    for (double v : k) sum += v;
    sum = 1.0 / sum;
    for (double& v : k) v = v * sum;
    return k;
}

// convolveLine(..., BORDER_TREATMENT_REFLECT): out[x] = float(sum_{p=x-r}^{x+r} k[x-p] * in[refl(p)])
// (internalConvolveLineReflect; the order of the additions is ascending p)
void convolve_line_reflect(const float* in, int64_t w, const std::vector<double>& k, float* out,
                           int64_t ostride) {
    int r = (int)(k.size() / 2);
    if (w < r + 1) throw std::runtime_error("convolveLine(): kernel longer than line");
    for (int64_t x = 0; x < w; ++x) {
        double sum = 0.0;
        for (int64_t p = x - r; p <= x + r; ++p) {
            int64_t q = p < 0 ? -p : (p >= w ? 2 * (w - 1) - p : p);
            double kv = k[(size_t)(r + (x - p))];
            sum += kv * (double)in[q];
        }
        out[x * ostride] = (float)sum;
    }
}

void gaussian_smoothing(const float* in, const Dims& d, const double* sigmas, float* out) {
    std::vector<float> line;
    if (out != in) std::memcpy(out, in, sizeof(float) * d.size);
    for (int k = 0; k < d.nd; ++k) {
        auto kern = gaussian_kernel(sigmas[k]);
        int64_t n = d.n[k], st = d.st[k];
        line.resize(n);
        for (int64_t base = 0; base < d.size; ++base) {
            int64_t c[3];
            coords(d, base, c);
            if (c[k] != 0) continue;
            for (int64_t i = 0; i < n; ++i) line[i] = out[base + i * st];
            convolve_line_reflect(line.data(), n, kern, out + base, st);
        }
    }
}

// ---------------------------------------------------------------------------------------
// localMaxima (2-D, 8-nbhd) / localMaxima3D (6-nbhd), allowPlateaus, allowAtBorder,
// threshold NumericTraits<float>::min() == -FLT_MAX.  out[i] = 1 for maxima voxels.
// ---------------------------------------------------------------------------------------
void local_maxima(const float* v, const Dims& d, uint8_t* out) {
    // neighbour deltas: 8 in 2-D, 6 in 3-D
    std::vector<std::array<int, 3>> deltas;
    if (d.nd == 2) deltas = indirect_deltas(2);
    else {
        for (auto& e : direct_nbrs(3)) {
            std::array<int, 3> a{0, 0, 0};
            a[e.dim] = e.sign;
            deltas.push_back(a);
        }
    }
    // plateau labelling with the same neighbourhood, equal values
    UF uf(d.size);
    int64_t c[3];
    for (int64_t i = 0; i < d.size; ++i) {
        coords(d, i, c);
        for (auto& a : deltas) {
            int64_t j = 0;
            bool ok = true;
            for (int k = 0; k < d.nd; ++k) {
                int64_t t = c[k] + a[k];
                if (t < 0 || t >= d.n[k]) { ok = false; break; }
                j += t * d.st[k];
            }
            if (ok && j < i && v[j] == v[i]) uf.unite(i, j);
        }
    }
    std::vector<uint8_t> is_ext(d.size, 1);
    const float threshold = -FLT_MAX;
    for (int64_t i = 0; i < d.size; ++i) {
        int64_t r = uf.find(i);
        if (!is_ext[r]) continue;
        if (!(v[i] > threshold)) { is_ext[r] = 0; continue; }
        coords(d, i, c);
        for (auto& a : deltas) {
            int64_t j = 0;
            bool ok = true;
            for (int k = 0; k < d.nd; ++k) {
                int64_t t = c[k] + a[k];
                if (t < 0 || t >= d.n[k]) { ok = false; break; }
                j += t * d.st[k];
            }
            if (ok && v[j] > v[i] && uf.find(j) != r) { is_ext[r] = 0; break; }
        }
    }
    for (int64_t i = 0; i < d.size; ++i) out[i] = is_ext[uf.find(i)] ? 1 : 0;
}

// strict local minima with the direct neighbourhood (vigra localMinMaxGraph, std::less,
// threshold FLT_MAX, allowAtBorder) -- the automatic seeds watershedsNew computes when
// the seed image is all zero (WatershedOptions: labels.any() == false).
void local_minima_strict(const float* v, const Dims& d, uint8_t* out) {
    auto nb = direct_nbrs(d.nd);
    int64_t c[3];
    for (int64_t i = 0; i < d.size; ++i) {
        out[i] = 0;
        if (!(v[i] < FLT_MAX)) continue;
        coords(d, i, c);
        bool mn = true;
        for (auto& e : nb) {
            int64_t t = c[e.dim] + e.sign;
            if (t < 0 || t >= d.n[e.dim]) continue;
            int64_t j = i + e.sign * d.st[e.dim];
            if (!(v[i] < v[j])) { mn = false; break; }
        }
        out[i] = mn ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------------------
// watershedsNew(image, seeds=labels) -> seededWatersheds (RegionGrowing, CompleteGrow).
// labels: in = seeds, out = result.  Returns maxRegionLabel.
// ---------------------------------------------------------------------------------------
struct PQCompare {
    bool operator()(const std::pair<int64_t, float>& l, const std::pair<int64_t, float>& r) const {
        return std::greater<float>()(l.second, r.second);
    }
};

// ---------------------------------------------------------------------------------------
// Model of the GPU flood (cluster_tools_amd/csrc/k_flood.hip): the same label-on-push
// region growing, but the priority is the total order key K = (C, d) then the label, with
// C the minimax height (float bits, order-preserving) and d the hop distance inside an
// equal-C plateau (g_tie_order 1; the other orders are the tie-order experiment's).  vigra breaks equal-C ties by heap position instead; this model is what
// the GPU must reproduce bit for bit, and VI(model, vigra) is the tie-break gap.
// ---------------------------------------------------------------------------------------
int g_flood_model = 0;
// tie orders for the tie-order experiment (scripts/tie_order_experiment.py): the GPU's
// order is 1 (unbounded d; the packed key's 12-bit field reports kDMax, cluster_tools_amd/csrc/ctws_dev.h).  Orders 2 and 6 have no
// unique fixpoint (equal keys along plateau paths), so no parallel relaxation can promise them.  2: (C, label), no hop distance; 3: (C, d, -label); 4: (C, d, push count) = FIFO
// inside an equal-(C, d) front; 5: (C, push count) = FIFO on a plateau; 6: (C, min(d, 1), label);
// 7: (C, label, d) -- the label before the hop distance; the fixpoint is unique, but a parallel
// relaxation does not reach it: round 5 on the GPU, a label whose source's C later drops stays
// on as a phantom whose d counts up to the saturation (count to infinity), DESIGN §4
int g_tie_order = 1;

inline uint32_t ordf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct ModelEntry {
    uint64_t key;
    uint32_t label;
    int64_t node;
    uint64_t seq;  // push count (tie orders 4, 5)
};
struct ModelCompare {
    bool operator()(const ModelEntry& a, const ModelEntry& b) const {
        if (g_tie_order == 7) {  // (C, label, d)
            const uint32_t ca = (uint32_t)(a.key >> 32), cb = (uint32_t)(b.key >> 32);
            if (ca != cb) return ca > cb;
            if (a.label != b.label) return a.label > b.label;
            return (a.key & 0xFFFFFFFFull) > (b.key & 0xFFFFFFFFull);
        }
        if (a.key != b.key) return a.key > b.key;
        switch (g_tie_order) {
            case 3: return a.label < b.label;
            case 4:
            case 5: return a.seq > b.seq;
            default: return a.label > b.label;
        }
    }
};

uint32_t watersheds_model(const float* h, const Dims& d, uint32_t* labels) {
    auto nb = direct_nbrs(d.nd);
    std::priority_queue<ModelEntry, std::vector<ModelEntry>, ModelCompare> pq;
    uint32_t maxRegionLabel = 0;
    uint64_t seq = 0;
    const bool use_d = g_tie_order != 2 && g_tie_order != 5;
    for (int64_t i = 0; i < d.size; ++i)
        if (labels[i]) {
            maxRegionLabel = std::max(maxRegionLabel, labels[i]);
            pq.push({(uint64_t)ordf(h[i]) << 32, labels[i], i, seq++});
        }
    int64_t c[3];
    while (!pq.empty()) {
        const ModelEntry e = pq.top();
        pq.pop();
        coords(d, e.node, c);
        for (auto& nbv : nb) {
            int64_t t = c[nbv.dim] + nbv.sign;
            if (t < 0 || t >= d.n[nbv.dim]) continue;
            int64_t j = e.node + nbv.sign * d.st[nbv.dim];
            if (labels[j] == 0) {
                labels[j] = e.label;
                const uint32_t hb = ordf(h[j]);
                const uint32_t cc = (uint32_t)(e.key >> 32);
                // d is unbounded (32 bits) in the GPU's order: the packed 12-bit d reports a
                // saturation and the GPU floods such a block again on wide keys (round 6);
                // order 6 caps it at 1
                const uint64_t dcap = g_tie_order == 6 ? 1ull : 0xFFFFFFFFull;
                const uint64_t k = hb > cc ? ((uint64_t)hb << 32)
                                           : (!use_d || (e.key & 0xFFFFFFFFull) >= dcap ? e.key : e.key + 1ull);
                pq.push({k, e.label, j, seq++});
            }
        }
    }
    return maxRegionLabel;
}

uint32_t watersheds_new(const float* h, const Dims& d, uint32_t* labels) {
    bool any = false;
    for (int64_t i = 0; i < d.size && !any; ++i) any = labels[i] != 0;
    if (!any) {
        // generateWatershedSeeds(..., SeedOptions() == Minima) + labelGraphWithBackground
        std::vector<uint8_t> mn(d.size);
        local_minima_strict(h, d, mn.data());
        label_with_background<uint8_t>(mn.data(), d, (uint8_t)0, labels);
    }
    if (g_flood_model) return watersheds_model(h, d, labels);
    auto nb = direct_nbrs(d.nd);
    std::priority_queue<std::pair<int64_t, float>, std::vector<std::pair<int64_t, float>>, PQCompare> pq;
    uint32_t maxRegionLabel = 0;
    int64_t c[3];
    scan_order(d, [&](int64_t i) {
        uint32_t lab = labels[i];
        if (lab == 0) return;
        if (maxRegionLabel < lab) maxRegionLabel = lab;
        coords(d, i, c);
        for (auto& e : nb) {
            int64_t t = c[e.dim] + e.sign;
            if (t < 0 || t >= d.n[e.dim]) continue;
            int64_t j = i + e.sign * d.st[e.dim];
            if (labels[j] == 0) {
                pq.push({i, h[i]});
                break;
            }
        }
    });
    while (!pq.empty()) {
        int64_t i = pq.top().first;
        float cost = pq.top().second;
        pq.pop();
        uint32_t lab = labels[i];
        coords(d, i, c);
        for (auto& e : nb) {
            int64_t t = c[e.dim] + e.sign;
            if (t < 0 || t >= d.n[e.dim]) continue;
            int64_t j = i + e.sign * d.st[e.dim];
            if (labels[j] == 0) {
                labels[j] = lab;
                float prio = std::max(h[j], cost);
                pq.push({j, prio});
            }
        }
    }
    return maxRegionLabel;
}

// vu.apply_size_filter (volume_utils.py:131-139): zero ids with count < size_filter (minus
// `exclude`), regrow with watershedsNew.  Returns the regrow's max label.
uint32_t apply_size_filter(uint32_t* seg, const float* h, const Dims& d, int size_filter,
                           const std::unordered_set<uint64_t>* exclude) {
    std::unordered_map<uint32_t, int64_t> counts;
    for (int64_t i = 0; i < d.size; ++i) counts[seg[i]]++;
    std::unordered_set<uint32_t> filt;
    for (auto& kv : counts)
        if (kv.second < size_filter) {
            if (exclude && exclude->count((uint64_t)kv.first)) continue;
            filt.insert(kv.first);
        }
    for (int64_t i = 0; i < d.size; ++i)
        if (filt.count(seg[i])) seg[i] = 0;
    return watersheds_new(h, d, seg);
}

// vu.watershed (volume_utils.py:123-128)
uint32_t vu_watershed(const float* h, const Dims& d, uint32_t* seeds_inout, int size_filter,
                      const std::unordered_set<uint64_t>* exclude) {
    uint32_t max_id = watersheds_new(h, d, seeds_inout);
    if (size_filter > 0) max_id = apply_size_filter(seeds_inout, h, d, size_filter, exclude);
    return max_id;
}

// vu.normalize (volume_utils.py:113-120) on float32 data in place
void normalize_inplace(float* x, int64_t n) {
    if (n == 0) return;
    float mn = x[0];
    for (int64_t i = 1; i < n; ++i) mn = std::min(mn, x[i]);
    for (int64_t i = 0; i < n; ++i) x[i] -= mn;
    float mx = x[0];
    for (int64_t i = 1; i < n; ++i) mx = std::max(mx, x[i]);
    if (mx > 0)
        for (int64_t i = 0; i < n; ++i) x[i] /= mx;
}

// watershed.py:163-169
void make_hmap(const float* input, const float* dt, int64_t n, const ctws_cfg& cfg, const Dims& d,
               float* hmap) {
    std::vector<float> dist(dt, dt + n);
    normalize_inplace(dist.data(), n);
    const float a = (float)cfg.alpha;
    const float b = (float)(1.0 - cfg.alpha);
    for (int64_t i = 0; i < n; ++i) {
        float di = 1.0f - dist[i];
        hmap[i] = a * input[i] + b * di;
    }
    bool smooth = cfg.sigma_weights_is_list ? true : (cfg.sigma_weights[0] != 0.0);
    if (smooth) {
        double s[3];
        if (cfg.sigma_weights_is_list) {
            if (d.nd != 3) throw std::runtime_error("apply_filter: len(sigma) != ndim");
            for (int k = 0; k < 3; ++k) s[k] = cfg.sigma_weights[k];
        } else {
            for (int k = 0; k < 3; ++k) s[k] = cfg.sigma_weights[0];
        }
        gaussian_smoothing(hmap, d, s, hmap);
    }
}

// watershed.py:179-207 (NMS branch unavailable: nifty.filters is not importable, :20-23)
void make_seeds(const float* dt, const Dims& d, const ctws_cfg& cfg, uint32_t* seeds) {
    std::vector<float> sm;
    const float* src = dt;
    bool smooth = cfg.sigma_seeds_is_list ? true : (cfg.sigma_seeds[0] != 0.0);
    if (smooth) {
        double s[3];
        if (cfg.sigma_seeds_is_list) {
            if (d.nd != 3) throw std::runtime_error("apply_filter: len(sigma) != ndim");
            for (int k = 0; k < 3; ++k) s[k] = cfg.sigma_seeds[k];
        } else {
            for (int k = 0; k < 3; ++k) s[k] = cfg.sigma_seeds[0];
        }
        sm.resize(d.size);
        gaussian_smoothing(dt, d, s, sm.data());
        src = sm.data();
    }
    std::vector<uint8_t> mx(d.size);
    local_maxima(src, d, mx.data());
    int64_t cnt = 0;
    for (int64_t i = 0; i < d.size; ++i) cnt += mx[i];
    if (cnt == d.size) {
        for (int64_t i = 0; i < d.size; ++i) seeds[i] = 1;
        return;
    }
    label_with_background<uint8_t>(mx.data(), d, (uint8_t)0, seeds);
}

// _read_data + normalize (watershed.py:267-282)
void read_data(const ctws_cfg& cfg, const ctws_block& b, std::vector<float>& out) {
    const int64_t n = b.outer_shape[0] * b.outer_shape[1] * b.outer_shape[2];
    auto load = [&](int64_t i) -> float {
        switch (b.input_dtype) {
            case CTWS_U8: return (float)((const uint8_t*)b.input)[i];
            case CTWS_U16: return (float)((const uint16_t*)b.input)[i];
            case CTWS_F32: return ((const float*)b.input)[i];
            case CTWS_F64: return (float)((const double*)b.input)[i];
        }
        throw std::runtime_error("bad dtype");
    };
    out.assign(n, 0.0f);
    if (b.n_channels > 0) {
        int64_t cb = cfg.channel_begin, ce = cfg.channel_end < 0 ? b.n_channels : cfg.channel_end;
        // python slice semantics for non-negative bounds
        if (cb < 0) cb += b.n_channels;
        if (ce > b.n_channels) ce = b.n_channels;
        if (cb > ce) cb = ce;
        int64_t C = ce - cb;
        if (C <= 0) throw std::runtime_error("empty channel range");
        std::vector<float> x(C * n);
        for (int64_t c = 0; c < C; ++c)
            for (int64_t i = 0; i < n; ++i) x[c * n + i] = load((cb + c) * n + i);
        normalize_inplace(x.data(), C * n);
        for (int64_t i = 0; i < n; ++i) {
            float acc = x[i];
            for (int64_t c = 1; c < C; ++c) {
                float v = x[c * n + i];
                if (cfg.agglomerate_channels == CTWS_AGG_MEAN) acc = acc + v;
                else if (cfg.agglomerate_channels == CTWS_AGG_MAX) acc = std::max(acc, v);
                else acc = std::min(acc, v);
            }
            if (cfg.agglomerate_channels == CTWS_AGG_MEAN) acc = acc / (float)C;
            out[i] = acc;
        }
    } else {
        for (int64_t i = 0; i < n; ++i) out[i] = load(i);
        normalize_inplace(out.data(), n);
    }
    if (cfg.invert_inputs)
        for (int64_t i = 0; i < n; ++i) out[i] = 1.0f - out[i];
}

// _apply_dt (watershed.py:139-160).  Returns false if nothing is above the threshold.
bool apply_dt(const std::vector<float>& input, const int64_t* shape, const ctws_cfg& cfg,
              std::vector<float>& dt) {
    const int64_t n = shape[0] * shape[1] * shape[2];
    const float thr = (float)cfg.threshold;
    std::vector<uint8_t> t(n);
    int64_t s = 0;
    for (int64_t i = 0; i < n; ++i) {
        t[i] = input[i] > thr;
        s += t[i];
    }
    if (s == 0) return false;
    dt.assign(n, 0.0f);
    if (cfg.apply_dt_2d) {
        if (cfg.has_pixel_pitch) throw std::runtime_error("apply_dt_2d requires pixel_pitch None");
        Dims d2 = make_dims(2, shape + 1);
        int64_t sl = shape[1] * shape[2];
        for (int64_t z = 0; z < shape[0]; ++z)
            distance_transform(t.data() + z * sl, d2, nullptr, dt.data() + z * sl);
    } else {
        Dims d3 = make_dims(3, shape);
        distance_transform(t.data(), d3, cfg.has_pixel_pitch ? cfg.pixel_pitch : nullptr, dt.data());
    }
    return true;
}

// _apply_watershed (watershed.py:211-249)
void apply_watershed(const std::vector<float>& input, std::vector<float>& dt, const int64_t* shape,
                     const ctws_cfg& cfg, const uint8_t* mask, std::vector<uint32_t>& ws) {
    const int64_t n = shape[0] * shape[1] * shape[2];
    ws.assign(n, 0);
    if (cfg.apply_ws_2d) {
        Dims d2 = make_dims(2, shape + 1);
        int64_t sl = shape[1] * shape[2];
        uint64_t offset = 0;
        std::vector<float> hm(sl);
        std::vector<uint32_t> wsz(sl);
        for (int64_t z = 0; z < shape[0]; ++z) {
            const float* dtz = dt.data() + z * sl;
            make_seeds(dtz, d2, cfg, wsz.data());
            make_hmap(input.data() + z * sl, dtz, sl, cfg, d2, hm.data());
            uint64_t max_id = vu_watershed(hm.data(), d2, wsz.data(), cfg.size_filter, nullptr);
            if (!mask) {
                for (int64_t i = 0; i < sl; ++i) wsz[i] = (uint32_t)(wsz[i] + offset);
            } else {
                const uint8_t* mz = mask + z * sl;
                uint64_t mx = 0;
                bool anym = false;
                for (int64_t i = 0; i < sl; ++i) {
                    if (!mz[i]) wsz[i] = 0;
                    else {
                        anym = true;
                        mx = std::max<uint64_t>(mx, wsz[i]);
                    }
                }
                max_id = anym ? mx : 0;
                for (int64_t i = 0; i < sl; ++i)
                    if (mz[i]) wsz[i] = (uint32_t)(wsz[i] + offset);
            }
            std::memcpy(ws.data() + z * sl, wsz.data(), sizeof(uint32_t) * sl);
            offset += max_id;
        }
    } else {
        Dims d3 = make_dims(3, shape);
        std::vector<float> hm(n);
        make_seeds(dt.data(), d3, cfg, ws.data());
        make_hmap(input.data(), dt.data(), n, cfg, d3, hm.data());
        vu_watershed(hm.data(), d3, ws.data(), cfg.size_filter, nullptr);
        if (mask)
            for (int64_t i = 0; i < n; ++i)
                if (!mask[i]) ws[i] = 0;
    }
}

// vigra relabelConsecutive(labels, start_label=1, keep_zeros=True) on uint32 labels
void relabel_consecutive(uint32_t* x, const Dims& d, std::unordered_map<uint32_t, uint32_t>& old_to_new) {
    old_to_new.clear();
    old_to_new[0] = 0;
    scan_order(d, [&](int64_t i) {
        auto it = old_to_new.find(x[i]);
        if (it != old_to_new.end()) {
            x[i] = it->second;
            return;
        }
        uint32_t nl = (uint32_t)(1 + old_to_new.size() - 1);
        old_to_new[x[i]] = nl;
        x[i] = nl;
    });
}

// two_pass_watershed.py:122-207.  inv_mask = voxels OUTSIDE the mask (NULL = no mask).
void apply_watershed_with_seeds(const std::vector<float>& input, std::vector<float>& dt,
                                const uint64_t* init, const int64_t* shape, const ctws_cfg& cfg,
                                const uint8_t* inv_mask, uint64_t offset, std::vector<uint64_t>& ws) {
    const int64_t n = shape[0] * shape[1] * shape[2];
    ws.assign(n, 0);
    if (cfg.apply_ws_2d) {
        Dims d2 = make_dims(2, shape + 1);
        int64_t sl = shape[1] * shape[2];
        std::vector<uint32_t> seeds(sl);
        std::vector<float> hm(sl);
        std::unordered_map<uint32_t, uint32_t> o2n;
        for (int64_t z = 0; z < shape[0]; ++z) {
            float* dtz = dt.data() + z * sl;
            const uint64_t* iz = init + z * sl;
            for (int64_t i = 0; i < sl; ++i)
                if (iz[i] != 0) dtz[i] = 0.0f;
            make_seeds(dtz, d2, cfg, seeds.data());
            if (inv_mask)
                for (int64_t i = 0; i < sl; ++i)
                    if (inv_mask[z * sl + i]) seeds[i] = 0;
            for (int64_t i = 0; i < sl; ++i)
                if (seeds[i] != 0) seeds[i] = (uint32_t)(seeds[i] + offset);  // uint32 wrap (B.2)
            for (int64_t i = 0; i < sl; ++i)
                if (iz[i] != 0) seeds[i] = (uint32_t)iz[i];  // setitem truncation (B.2)
            relabel_consecutive(seeds.data(), d2, o2n);
            std::unordered_map<uint32_t, uint32_t> n2o;
            for (auto& kv : o2n) n2o[kv.second] = kv.first;
            make_hmap(input.data() + z * sl, dtz, sl, cfg, d2, hm.data());
            std::unordered_set<uint64_t> excl(iz, iz + sl);  // exclude=initial_seeds_z (B.3)
            uint64_t max_id = vu_watershed(hm.data(), d2, seeds.data(), cfg.size_filter, &excl);
            if (inv_mask) {
                uint64_t mx = 0;
                bool any_in = false;
                for (int64_t i = 0; i < sl; ++i) {
                    if (inv_mask[z * sl + i]) seeds[i] = 0;
                    else {
                        any_in = true;
                        mx = std::max<uint64_t>(mx, seeds[i]);
                    }
                }
                max_id = any_in ? mx : 0;
            }
            offset += max_id;
            for (int64_t i = 0; i < sl; ++i) {
                auto it = n2o.find(seeds[i]);
                if (it == n2o.end()) throw std::runtime_error("takeDict: missing key");
                ws[z * sl + i] = it->second;
            }
        }
    } else {
        Dims d3 = make_dims(3, shape);
        std::vector<uint32_t> seeds(n);
        make_seeds(dt.data(), d3, cfg, seeds.data());
        if (inv_mask)
            for (int64_t i = 0; i < n; ++i)
                if (inv_mask[i]) seeds[i] = 0;
        for (int64_t i = 0; i < n; ++i)
            if (seeds[i] != 0) seeds[i] = (uint32_t)(seeds[i] + offset);
        std::unordered_set<uint64_t> excl;
        for (int64_t i = 0; i < n; ++i)
            if (init[i] != 0) {
                seeds[i] = (uint32_t)init[i];
                excl.insert(init[i]);
            }
        std::unordered_map<uint32_t, uint32_t> o2n;
        relabel_consecutive(seeds.data(), d3, o2n);
        std::unordered_map<uint32_t, uint32_t> n2o;
        for (auto& kv : o2n) n2o[kv.second] = kv.first;
        std::vector<float> hm(n);
        make_hmap(input.data(), dt.data(), n, cfg, d3, hm.data());
        vu_watershed(hm.data(), d3, seeds.data(), cfg.size_filter, &excl);
        for (int64_t i = 0; i < n; ++i) {
            auto it = n2o.find(seeds[i]);
            if (it == n2o.end()) throw std::runtime_error("takeDict: missing key");
            ws[i] = it->second;
        }
        if (inv_mask)
            for (int64_t i = 0; i < n; ++i)
                if (inv_mask[i]) ws[i] = 0;
    }
}

thread_local std::string g_err;

}  // namespace

// =========================================================================================
// C-ABI of the oracle (loaded by ctypes from tests/ and bench.py's cpu_baseline leg)
// =========================================================================================
extern "C" {

const char* orc_last_error() { return g_err.c_str(); }

// 0: vigra's heap order (the reference); 1: the GPU flood's (C, d, label) order (model)
void orc_set_flood_model(int on) { g_flood_model = on; }
void orc_set_tie_order(int order) { g_tie_order = order; }

// stage-level entry points (for cross-checks against scipy / scikit-image)
int orc_distance_transform(const uint8_t* fg, int nd, const int64_t* shape, const double* pitch,
                           float* out) {
    try {
        distance_transform(fg, make_dims(nd, shape), pitch, out);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int orc_gaussian_kernel(double sigma, double* taps, int max_taps) {
    auto k = gaussian_kernel(sigma);
    if ((int)k.size() > max_taps) return -1;
    for (size_t i = 0; i < k.size(); ++i) taps[i] = k[i];
    return (int)k.size();
}

int orc_gaussian_smoothing(const float* in, int nd, const int64_t* shape, const double* sigmas,
                           float* out) {
    try {
        gaussian_smoothing(in, make_dims(nd, shape), sigmas, out);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int orc_local_maxima(const float* in, int nd, const int64_t* shape, uint8_t* out) {
    local_maxima(in, make_dims(nd, shape), out);
    return 0;
}

int64_t orc_label_u8(const uint8_t* in, int nd, const int64_t* shape, uint32_t* out) {
    return label_with_background<uint8_t>(in, make_dims(nd, shape), 0, out);
}

int64_t orc_label_u32(const uint32_t* in, int nd, const int64_t* shape, uint32_t* out) {
    return label_with_background<uint32_t>(in, make_dims(nd, shape), 0u, out);
}

int64_t orc_watershed(const float* h, int nd, const int64_t* shape, uint32_t* labels) {
    return watersheds_new(h, make_dims(nd, shape), labels);
}

int64_t orc_make_seeds(const float* dt, int nd, const int64_t* shape, const ctws_cfg* cfg,
                       uint32_t* seeds) {
    try {
        make_seeds(dt, make_dims(nd, shape), *cfg, seeds);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int orc_make_hmap(const float* input, const float* dt, int nd, const int64_t* shape,
                  const ctws_cfg* cfg, float* hmap) {
    try {
        Dims d = make_dims(nd, shape);
        make_hmap(input, dt, d.size, *cfg, d, hmap);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Intermediate stages of the last orc_ws_block call (outer-shaped), for fixtures.
struct OrcStages {
    float* input;   // normalized input (after invert / mask)
    float* dt;      // distance transform (NULL-safe)
    uint32_t* ws;   // uint32 watershed before crop (outer shaped)
};

// _ws_block / _ws_pass2 for each block: same contract as ctws_ws_blocks with host pointers.
int orc_ws_blocks(const ctws_cfg* cfg, ctws_block* blocks, int n_blocks, OrcStages* stages) {
    try {
        if (cfg->non_maximum_suppression) {
            // watershed.py:182-184 logs "not available" and continues without NMS
        }
        for (int bi = 0; bi < n_blocks; ++bi) {
            ctws_block& b = blocks[bi];
            const int64_t* sh = b.outer_shape;
            const int64_t n = sh[0] * sh[1] * sh[2];
            const int64_t* ib = b.inner_begin;
            const int64_t* is = b.inner_shape;
            const int64_t ni = is[0] * is[1] * is[2];
            auto inner_idx = [&](int64_t z, int64_t y, int64_t x) {
                return ((z + ib[0]) * sh[1] + (y + ib[1])) * sh[2] + (x + ib[2]);
            };
            b.status = CTWS_BLOCK_WRITTEN;
            b.max_label = 0;
            // mask: skip if the inner mask is empty (watershed.py:290-297)
            if (b.mask) {
                int64_t s = 0;
                for (int64_t z = 0; z < is[0]; ++z)
                    for (int64_t y = 0; y < is[1]; ++y)
                        for (int64_t x = 0; x < is[2]; ++x) s += b.mask[inner_idx(z, y, x)] != 0;
                if (s == 0) {
                    b.status = CTWS_BLOCK_SKIPPED_MASK;
                    continue;
                }
            }
            std::vector<float> input;
            read_data(*cfg, b, input);
            if (b.mask)
                for (int64_t i = 0; i < n; ++i)
                    if (!b.mask[i]) input[i] = 1.0f;
            const uint64_t offset = (uint64_t)b.block_id *
                                    (uint64_t)(cfg->block_shape[0] * cfg->block_shape[1] * cfg->block_shape[2]);
            std::vector<float> dt;
            bool ok = apply_dt(input, sh, *cfg, dt);
            if (stages) {
                std::memcpy(stages[bi].input, input.data(), sizeof(float) * n);
                if (ok) std::memcpy(stages[bi].dt, dt.data(), sizeof(float) * n);
                else std::memset(stages[bi].dt, 0, sizeof(float) * n);
            }
            if (cfg->pass_id == 1) {
                // _ws_pass2 (two_pass_watershed.py:210-255)
                if (!ok) {
                    b.status = CTWS_BLOCK_EMPTY_PASS2;
                    continue;
                }
                std::vector<uint8_t> inv;
                if (b.mask) {
                    inv.resize(n);
                    for (int64_t i = 0; i < n; ++i) inv[i] = b.mask[i] == 0;
                }
                std::vector<uint64_t> ws;
                apply_watershed_with_seeds(input, dt, b.initial_seeds, sh, *cfg, b.mask ? inv.data() : nullptr,
                                           offset, ws);
                uint64_t mx = 0;
                for (int64_t z = 0; z < is[0]; ++z)
                    for (int64_t y = 0; y < is[1]; ++y)
                        for (int64_t x = 0; x < is[2]; ++x) {
                            uint64_t v = ws[inner_idx(z, y, x)];
                            b.output[(z * is[1] + y) * is[2] + x] = v;
                            mx = std::max(mx, v);
                        }
                b.max_label = mx;
                if (stages)
                    for (int64_t i = 0; i < n; ++i) stages[bi].ws[i] = (uint32_t)ws[i];
                continue;
            }
            if (!ok) {
                // watershed.py:310-321: constant offset, masked voxels 0
                b.status = CTWS_BLOCK_EMPTY;
                for (int64_t z = 0; z < is[0]; ++z)
                    for (int64_t y = 0; y < is[1]; ++y)
                        for (int64_t x = 0; x < is[2]; ++x) {
                            bool in = !b.mask || b.mask[inner_idx(z, y, x)];
                            b.output[(z * is[1] + y) * is[2] + x] = in ? offset : 0;
                        }
                if (stages) std::memset(stages[bi].ws, 0, sizeof(uint32_t) * n);
                continue;
            }
            std::vector<uint32_t> ws;
            apply_watershed(input, dt, sh, *cfg, b.mask, ws);
            if (stages) std::memcpy(stages[bi].ws, ws.data(), sizeof(uint32_t) * n);
            std::vector<uint32_t> res(ni);
            std::vector<uint8_t> inm;
            if (b.crop_relabel) {
                std::vector<uint32_t> crop(ni);
                for (int64_t z = 0; z < is[0]; ++z)
                    for (int64_t y = 0; y < is[1]; ++y)
                        for (int64_t x = 0; x < is[2]; ++x)
                            crop[(z * is[1] + y) * is[2] + x] = ws[inner_idx(z, y, x)];
                label_with_background<uint32_t>(crop.data(), make_dims(3, is), 0u, res.data());
                if (b.mask) {
                    inm.resize(ni);
                    for (int64_t z = 0; z < is[0]; ++z)
                        for (int64_t y = 0; y < is[1]; ++y)
                            for (int64_t x = 0; x < is[2]; ++x)
                                inm[(z * is[1] + y) * is[2] + x] = b.mask[inner_idx(z, y, x)] != 0;
                }
            } else {
                // output_bb == input_bb: the inner block is the outer block
                for (int64_t i = 0; i < ni; ++i) res[i] = ws[i];
                if (b.mask) {
                    inm.resize(ni);
                    for (int64_t i = 0; i < ni; ++i) inm[i] = b.mask[i] != 0;
                }
            }
            uint64_t mx = 0;
            for (int64_t i = 0; i < ni; ++i) {
                uint64_t v = res[i];
                mx = std::max(mx, v);
                if (!b.mask || inm[i]) v += offset;
                b.output[i] = v;
            }
            b.max_label = mx;
        }
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// WatershedFromSeeds `_ws_block` / `_ws_block_masked` (watershed/watershed_from_seeds.py:
// 143-199) for each block: no halo (input = output = the block), `_read_data` (:125-140:
// normalize, 4-D channel agglomeration, no invert), seeds = ds_seeds[bb] as uint32 after the
// `max_id < uint32 max` assert (:160-163; a block failing it gets CTWS_BLOCK_FAILED),
// vu.watershed(input, seeds, size_filter) (3-D, direct nbhd), masked voxels: input 1 before,
// label 0 after the flood (:186-198); an empty block mask writes nothing (:178-181).
int orc_ws_from_seeds(const ctws_cfg* cfg_in, ctws_block* blocks, int n_blocks) {
    try {
        ctws_cfg cfg = *cfg_in;
        cfg.invert_inputs = 0;
        for (int bi = 0; bi < n_blocks; ++bi) {
            ctws_block& b = blocks[bi];
            const int64_t* sh = b.outer_shape;
            const int64_t n = sh[0] * sh[1] * sh[2];
            b.status = CTWS_BLOCK_WRITTEN;
            b.max_label = 0;
            if (b.mask) {
                int64_t s = 0;
                for (int64_t i = 0; i < n; ++i) s += b.mask[i] != 0;
                if (s == 0) {
                    b.status = CTWS_BLOCK_SKIPPED_MASK;
                    continue;
                }
            }
            uint64_t smax = 0;
            for (int64_t i = 0; i < n; ++i) smax = std::max(smax, b.initial_seeds[i]);
            if (smax >= 0xFFFFFFFFull) {
                b.status = CTWS_BLOCK_FAILED;  // AssertionError "Overflow detected"
                continue;
            }
            std::vector<float> input;
            read_data(cfg, b, input);
            if (b.mask)
                for (int64_t i = 0; i < n; ++i)
                    if (!b.mask[i]) input[i] = 1.0f;
            std::vector<uint32_t> ws(n);
            for (int64_t i = 0; i < n; ++i) ws[i] = (uint32_t)b.initial_seeds[i];
            const uint32_t mx = vu_watershed(input.data(), make_dims(3, sh), ws.data(), cfg.size_filter, nullptr);
            for (int64_t i = 0; i < n; ++i) b.output[i] = (b.mask && !b.mask[i]) ? 0ull : (uint64_t)ws[i];
            b.max_label = mx;
        }
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

}  // extern "C"
