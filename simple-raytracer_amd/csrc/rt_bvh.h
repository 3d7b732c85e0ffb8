// rt_bvh.h -- host-side BVH builder for the MI355X renderer (header-only,
// included by rt_kernels.hip's host code).
//
// The reference scans every primitive for every ray (TraceRay, main.cpp:1218-
// 1403).  The BVH only decides WHICH primitives a ray can possibly hit; every
// candidate is still tested with the reference's exact formulas, and the
// device traversal answers the reference's order-dependent cases exactly
// (closest-hit ties, SKIP_TRANS).  For that the boxes must
// be conservative for the *computed* intersections, which deviate from exact
// geometry by rounding (build_bvh in rt_kernels.hip pads the primitives):
//   face:   the accepted hit point is within a few ulp(scene scale) of the
//           triangle -> pad by 2^-16 * D * max(1, cond), cond = |e1|^2|e2|^2/det
//           (32x the rounding bound of the barycentric test)
//   sphere: the discriminant B^2 - 4C is computed with absolute error up to
//           ~2^-18.4 D^2 (|dir| <= D), so rays up to sqrt(r^2 + 2^-20 D^2) from
//           the centre can be "hits" -> radius grown to sqrt(r^2 + 2^-18 D^2)
//           + 2^-16 D (a factor 4 of margin on the error term)
// where D bounds the distance from any ray origin (eye or a surface point) to
// any primitive.  (The directional-light sphere quirk -- A = 1 assumed for an
// unnormalised direction -- is not ray geometry: those shadow rays query a
// per-light cone tree over the spheres, dir_tree in rt_kernels.hip.)
#pragma once

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

namespace rtbvh {

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY};
    float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box &b) {
        for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], b.lo[k]), hi[k] = std::max(hi[k], b.hi[k]);
    }
    void grow(const float p[3]) {
        for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], p[k]), hi[k] = std::max(hi[k], p[k]);
    }
    float area() const {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0f;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

// 64-byte node: both children's boxes + child links.  link >= 0: inner node
// index; link < 0: leaf, -(1 + (first << 4 | count)), count <= 15.
struct Node {
    float l_lo[3], l_hi0;
    float l_hi12[2], r_lo01[2];
    float r_lo2, r_hi[3];
    int32_t link[2];
    int32_t pad[2];
};
static_assert(sizeof(Node) == 64, "node layout");

struct Prim {
    Box box;
    float c[3];
    float cost;   // relative intersection cost
    int key;      // object index (reference visiting order)
};

struct Result {
    std::vector<Node> nodes;
    std::vector<int32_t> keys;   // leaf-ordered object indices
    std::vector<float> costs;    // their Prim::cost
    int depth = 0;
};

inline int32_t leaf_link(int first, int count) { return -(1 + ((first << 4) | count)); }

// W-wide node (W = 4: 128 B, W = 8: 240 B; host-side form): the children's
// boxes as SoA rows + links.  Unused slots carry link kEmpty.  Built by
// collapsing the binary tree (each node absorbs grandchildren, largest surface
// area first).
constexpr int32_t kEmpty = INT32_MIN;
// Device form of an unused slot: a leaf with no primitives (leaf_records'
// encoding with offset 0, count 0), so the traversal needs no link test.
constexpr int32_t kEmptyLeaf = -1;
template <int W>
struct NodeW {
    float lo[3][W];
    float hi[3][W];
    int32_t link[W];
    int32_t max_stack;       // worst-case traversal stack entries below (root only)
    int32_t pad[3];
};
using Node4 = NodeW<4>;
static_assert(sizeof(Node4) == 128, "node4 layout");

template <int W>
struct ResultW {
    std::vector<NodeW<W>> nodes;
    int depth = 0;
    int max_stack = 0;       // worst-case entries a near-first traversal pushes
};
using Result4 = ResultW<4>;

// Collapse a binary tree (Result) into W-wide nodes.
template <int W>
inline void collapse(const Result &R, ResultW<W> &Q) {
    Q = ResultW<W>();
    if (R.nodes.empty()) return;
    struct Child {
        int32_t link;
        Box box;
    };
    auto children2 = [&](int ni, Child out[2]) {
        const Node &n = R.nodes[ni];
        out[0].link = n.link[0];
        out[1].link = n.link[1];
        for (int k = 0; k < 3; k++) out[0].box.lo[k] = n.l_lo[k];
        out[0].box.hi[0] = n.l_hi0, out[0].box.hi[1] = n.l_hi12[0], out[0].box.hi[2] = n.l_hi12[1];
        out[1].box.lo[0] = n.r_lo01[0], out[1].box.lo[1] = n.r_lo01[1], out[1].box.lo[2] = n.r_lo2;
        for (int k = 0; k < 3; k++) out[1].box.hi[k] = n.r_hi[k];
    };
    // returns the node index; `stack_in` = entries already on the stack on entry
    std::function<int(int, int, int)> conv = [&](int ni, int depth, int stack_in) -> int {
        Child ch[W];
        int n = 2;
        children2(ni, ch);
        for (;;) {
            if (n == W) break;
            int best = -1;
            float ba = -1;
            for (int i = 0; i < n; i++)
                if (ch[i].link >= 0 && ch[i].box.area() > ba) ba = ch[i].box.area(), best = i;
            if (best < 0) break;
            Child g[2];
            children2(ch[best].link, g);
            ch[best] = g[0];
            ch[n++] = g[1];
        }
        int qi = (int)Q.nodes.size();
        Q.nodes.emplace_back();
        Q.depth = std::max(Q.depth, depth);
        // near-first traversal: visiting a child keeps up to (hits - 1) siblings on the stack
        int below = stack_in + (n - 1);
        Q.max_stack = std::max(Q.max_stack, below);
        int32_t links[W];
        for (int i = 0; i < W; i++) links[i] = kEmpty;
        for (int i = 0; i < n; i++) links[i] = ch[i].link >= 0 ? conv(ch[i].link, depth + 1, below) : ch[i].link;
        NodeW<W> &q = Q.nodes[qi];
        for (int i = 0; i < W; i++) {
            for (int k = 0; k < 3; k++) {
                q.lo[k][i] = i < n ? ch[i].box.lo[k] : INFINITY;
                q.hi[k][i] = i < n ? ch[i].box.hi[k] : -INFINITY;
            }
            q.link[i] = links[i];
        }
        q.max_stack = 0;
        q.pad[0] = q.pad[1] = q.pad[2] = 0;
        return qi;
    };
    conv(0, 1, 0);
    Q.nodes[0].max_stack = Q.max_stack;
}

// SAH-optimal collapse (Ylitie et al. 2017, §3.1).  Over the binary tree,
// C(n, i) is the least SAH cost of covering subtree n with at most i units,
// each unit a leaf (<= max_leaf primitives) or a W-wide node:
//   C(n, 1) = min(leaf: A(n) * sum(cost), node: A(n) * node_cost + dist(n, W))
//   C(n, i) = min(C(n, i - 1), dist(n, i))
//   dist(n, j) = min over k of C(left, k) + C(right, j - k)
// (costs in primitive tests, A = surface area).  The binary tree should go
// down to single primitives (Builder::max_leaf = 1): the DP picks the leaves.
template <int W>
inline void collapse_sah(const Result &R, ResultW<W> &Q, int max_leaf, float node_cost) {
    Q = ResultW<W>();
    if (R.nodes.empty()) return;
    const int ni_count = (int)R.nodes.size();
    struct Ref {
        int32_t link;
        Box box;
    };
    auto kids = [&](int ni, Ref out[2]) {
        const Node &n = R.nodes[ni];
        out[0].link = n.link[0];
        out[1].link = n.link[1];
        for (int k = 0; k < 3; k++) out[0].box.lo[k] = n.l_lo[k];
        out[0].box.hi[0] = n.l_hi0, out[0].box.hi[1] = n.l_hi12[0], out[0].box.hi[2] = n.l_hi12[1];
        out[1].box.lo[0] = n.r_lo01[0], out[1].box.lo[1] = n.r_lo01[1], out[1].box.lo[2] = n.r_lo2;
        for (int k = 0; k < 3; k++) out[1].box.hi[k] = n.r_hi[k];
    };
    auto leaf_sum = [&](int32_t link, int &first, int &count) {
        int v = -link - 1;
        first = v >> 4, count = v & 15;
        float s = 0;
        for (int i = first; i < first + count; i++) s += R.costs[i];
        return s;
    };
    std::vector<int> first(ni_count, 0), cnt(ni_count, 0);
    std::vector<float> psum(ni_count, 0.0f);
    std::vector<float> C((size_t)ni_count * (W + 1), 0.0f);
    std::vector<int8_t> D((size_t)ni_count * (W + 1), 0);   // i = 1: 0 leaf / k; i > 1: 0 "as i - 1" / k
    auto cost = [&](const Ref &r, int i) -> float {
        if (r.link >= 0) return C[(size_t)r.link * (W + 1) + i];
        int f, c;
        return r.box.area() * leaf_sum(r.link, f, c);
    };
    // children have larger indices than their parent (Builder::build_range)
    for (int n = ni_count - 1; n >= 0; n--) {
        Ref ch[2];
        kids(n, ch);
        Box b = ch[0].box;
        b.grow(ch[1].box);
        const float A = b.area();
        int lo = INT32_MAX, num = 0;
        float s = 0;
        for (const Ref &r : ch) {
            int f, c;
            if (r.link >= 0) f = first[r.link], c = cnt[r.link], s += psum[r.link];
            else s += leaf_sum(r.link, f, c);
            if (c > 0) lo = std::min(lo, f);
            num += c;
        }
        first[n] = num > 0 ? lo : 0, cnt[n] = num, psum[n] = s;
        float *Cn = &C[(size_t)n * (W + 1)];
        int8_t *Dn = &D[(size_t)n * (W + 1)];
        // the children's costs as 1..W units, once (cost() of a leaf child
        // is its area times its primitives' cost, whatever the units)
        float cc[2][W + 1];
        for (int side = 0; side < 2; side++)
            for (int k = 1; k <= W; k++) cc[side][k] = (ch[side].link >= 0 || k == 1) ? cost(ch[side], k) : cc[side][1];
        auto dist = [&](int j, int &kbest) {
            float best = INFINITY;
            kbest = 1;
            for (int k = 1; k < j; k++) {
                float c = cc[0][k] + cc[1][j - k];
                if (c < best) best = c, kbest = k;
            }
            return best;
        };
        int kw;
        const float c_node = A * node_cost + dist(W, kw);
        const float c_leaf = (num <= max_leaf && num <= 15) ? A * s : INFINITY;
        if (c_leaf <= c_node) Cn[1] = c_leaf, Dn[1] = 0;
        else Cn[1] = c_node, Dn[1] = (int8_t)kw;
        for (int i = 2; i <= W; i++) {
            int k;
            float d = dist(i, k);
            if (d < Cn[i - 1]) Cn[i] = d, Dn[i] = (int8_t)k;
            else Cn[i] = Cn[i - 1], Dn[i] = 0;
        }
    }
    struct Units {                                    // at most W units of one node
        Ref r[W];
        int m = 0;
        void push_back(const Ref &x) { r[m++] = x; }
    };
    // subtree `r` as at most i units
    std::function<void(const Ref &, int, Units &)> gather = [&](const Ref &r, int i, Units &out) {
        if (r.link < 0) {
            out.push_back(r);
            return;
        }
        const int8_t *Dn = &D[(size_t)r.link * (W + 1)];
        while (i > 1 && Dn[i] == 0) i--;
        if (i == 1) {
            out.push_back(r);
            return;
        }
        Ref ch[2];
        kids(r.link, ch);
        gather(ch[0], Dn[i], out);
        gather(ch[1], i - Dn[i], out);
    };
    // one unit: a leaf link or a new W-wide node (the root is always a node)
    std::function<int32_t(const Ref &, int, int, bool)> emit = [&](const Ref &r, int depth, int stack_in,
                                                                   bool root) -> int32_t {
        if (r.link < 0) return r.link;
        const int n = r.link;
        int k = D[(size_t)n * (W + 1) + 1];
        if (k == 0 && !root) return leaf_link(first[n], cnt[n]);
        Ref ch2[2];
        kids(n, ch2);
        if (k == 0) {                                 // the root as a node although a leaf is cheaper
            float best = INFINITY;
            for (int j = 1; j < W; j++) {
                float c = cost(ch2[0], j) + cost(ch2[1], W - j);
                if (c < best) best = c, k = j;
            }
        }
        Units us;
        gather(ch2[0], k, us);
        gather(ch2[1], W - k, us);
        const Ref *ch = us.r;
        const int m = us.m;
        int qi = (int)Q.nodes.size();
        Q.nodes.emplace_back();
        Q.depth = std::max(Q.depth, depth);
        const int below = stack_in + (m - 1);
        Q.max_stack = std::max(Q.max_stack, below);
        int32_t links[W];
        for (int i = 0; i < W; i++) links[i] = kEmpty;
        for (int i = 0; i < m; i++) links[i] = emit(ch[i], depth + 1, below, false);
        NodeW<W> &q = Q.nodes[qi];
        for (int i = 0; i < W; i++) {
            for (int a = 0; a < 3; a++) {
                q.lo[a][i] = i < m ? ch[i].box.lo[a] : INFINITY;
                q.hi[a][i] = i < m ? ch[i].box.hi[a] : -INFINITY;
            }
            q.link[i] = links[i];
        }
        q.max_stack = 0;
        q.pad[0] = q.pad[1] = q.pad[2] = 0;
        return qi;
    };
    Ref root;
    root.link = 0;
    emit(root, 1, 0, true);
    Q.nodes[0].max_stack = Q.max_stack;
}

// Device form of a 4-wide node (104 B; after Ylitie et al. 2017,
// with half-precision instead of 8-bit plane offsets): the node's box origin,
// one power-of-two scale 2^e for the three axes (stored as the float 2^e: the
// device forms 2^e / d with one multiply per axis), each child's bounds as
// binary16 multiples h of it -- lower bounds rounded down, upper bounds rounded
// up, to the binary16 grid (child i in half i % 2 of word i / 2) -- then the
// links.  Child box on axis a: [origin_a + hlo * 2^e, origin_a + hhi * 2^e]; it
// contains the float box exactly (real arithmetic), and the device's
// slab-test rounding is of the order of ulp(D), far inside the primitives'
// padding (rt_kernels.hip).  The device converts h inside the plane FMA
// (v_fma_mix_f32): no separate conversion instruction per plane, and 2^-11
// relative resolution (8-bit offsets: 1/255) -- tighter boxes.
//
// Per axis the bounds are stored as lo(0,1) lo(2,3) hi(0,1) hi(2,3) lo(0,1)
// lo(2,3): the 16 bytes at word 0 are (lower, upper) and the 16 bytes at word
// 2 are (upper, lower) -- a ray reads the window that puts its near planes
// first (word 2 when its direction along the axis is negative), so the device
// selects near / far planes by a load offset, not by 4 v_cndmask per axis.
struct Node4H {
    float origin[3];
    float scale;             // 2^e (-126 <= e <= kQExpMax), one for the three axes
    uint32_t ax[3][6];       // per axis: lo(0,1) lo(2,3) hi(0,1) hi(2,3) lo(0,1) lo(2,3)
    int32_t link[4];
    uint32_t lo(int a, int j) const { return ax[a][j]; }
    uint32_t hi(int a, int j) const { return ax[a][2 + j]; }
};
static_assert(sizeof(Node4H) == 104, "node4 device layout");
constexpr int kNodeAxisOff = 16;         // byte offset of axis 0's words; axis a at 16 + 24 a
constexpr int kNodeLinkOff = 88;         // byte offset of the links

// h in [0, kHMax]: 2048 keeps the offsets where binary16 is integer-exact
constexpr double kHMax = 2048.0;
// Largest scale exponent: the device forms 2^e * (1/d) with |1/d| capped at
// 2^100, which stays finite for e <= 27 (node extents up to 2048 * 2^27).
constexpr int kQExpMax = 27;
// empty slot: an inverted box in every axis (lower bound kHMax, upper 0)
constexpr uint16_t kHalfHMax = 0x6800;   // 2048.0 in binary16

// bits of a non-negative double that is a binary16 value
inline uint16_t half_bits(double r) {
    if (!(r > 0)) return 0;
    int k;
    std::frexp(r, &k);                       // r in [2^(k-1), 2^k)
    const int E = k - 1;
    if (E < -14) return (uint16_t)std::ldexp(r, 24);                       // subnormal
    return (uint16_t)(((E + 15) << 10) | ((uint32_t)std::ldexp(r, 10 - E) - 1024u));
}
// the largest binary16 value <= v (up = false) or the smallest >= v (up =
// true), for v in [0, kHMax]: v = m * 2^u with u the binary16 ulp exponent
// of v's binade (2^-24 below 2^-14), m rounded down / up to an integer; a
// carry to m = 2^11 moves to the next binade.  Bit operations on the double:
// exact, and the same bits as the frexp / ldexp formulation (half_bits(m 2^u))
inline uint16_t half_round(double v, bool up) {
    if (!(v > 0)) return 0;
    uint64_t b;
    std::memcpy(&b, &v, sizeof b);
    const int E = (int)((b >> 52) & 0x7ff) - 1023;          // v normal: v in [2^E, 2^(E+1)), E <= 11
    const int u = std::max(E, -14) - 10;                     // ulp exponent
    // m = v / 2^u as a 53-bit fixed-point integer part: shift the significand
    const uint64_t sig = (b & ((uint64_t(1) << 52) - 1)) | (uint64_t(1) << 52);   // v = sig * 2^(E - 52)
    const int sh = 52 - (E - u);                             // v / 2^u = sig >> sh (sh >= 42 for u >= E - 10)
    uint64_t m;
    if (sh >= 64) {
        m = up ? 1 : 0;                                      // v < 2^u (v > 0): rounds to 0 or one ulp
    } else {
        m = sig >> sh;
        if (up && (sig & ((uint64_t(1) << sh) - 1))) m++;
    }
    int ue = u;
    if (m == 2048) m = 1024, ue++;                           // carry into the next binade
    if (m == 0) return 0;
    if (m < 1024) return (uint16_t)m;                        // subnormal (ue = -24)
    return (uint16_t)(((ue + 10 + 15) << 10) | (uint32_t)(m - 1024));
}
// value of binary16 bits (non-negative)
inline double half_value(uint16_t b) {
    const int E = (b >> 10) & 31, m = b & 1023;
    return E == 0 ? std::ldexp((double)m, -24) : std::ldexp(1024.0 + m, E - 25);
}

// Run f(begin, end) over [0, n) in `threads` contiguous slices (the
// results must not depend on the split).
template <class F>
inline void parallel_ranges(size_t n, int threads, F f) {
    const size_t t = (size_t)std::max(1, std::min<int>(threads, (int)((n + 2047) / 2048)));
    if (t <= 1) {
        f((size_t)0, n);
        return;
    }
    std::vector<std::thread> pool;
    for (size_t k = 1; k < t; k++) pool.emplace_back(f, n * k / t, n * (k + 1) / t);
    f((size_t)0, n / t);
    for (auto &th : pool) th.join();
}

// One node of quantize; false if a child box is not finite or the node is too
// large for kQExpMax.
inline bool quantize_node(const Node4 &n, Node4H &z) {
    z = Node4H{};
    for (int i = 0; i < 4; i++) z.link[i] = n.link[i];
    double lo[3], hi[3];
    int e = -126;
    for (int a = 0; a < 3; a++) {
        auto empty = [&](int i) {              // no slot, or an empty leaf (inverted box)
            return n.link[i] == kEmpty || !(n.lo[a][i] <= n.hi[a][i]);
        };
        lo[a] = INFINITY, hi[a] = -INFINITY;
        for (int i = 0; i < 4; i++) {
            if (empty(i)) continue;
            if (!std::isfinite(n.lo[a][i]) || !std::isfinite(n.hi[a][i])) return false;
            lo[a] = std::min(lo[a], (double)n.lo[a][i]);
            hi[a] = std::max(hi[a], (double)n.hi[a][i]);
        }
        if (!(lo[a] <= hi[a])) lo[a] = hi[a] = 0.0;  // no child at all
        z.origin[a] = (float)lo[a];                  // exact: lo is a float
        // smallest scale 2^e with kHMax * 2^e >= every axis' extent (normal
        // floats only); binary16 is floating point, so a shorter axis keeps
        // 11 significant bits in its offsets.  ext / kHMax = m 2^k with m in
        // [1/2, 1) (exact: a power-of-two division): 2^e >= it from e = k,
        // or k - 1 when m = 1/2
        const double ext = hi[a] - lo[a];
        if (ext > std::ldexp(kHMax, e)) {
            int k;
            const double m = std::frexp(ext / kHMax, &k);
            e = std::min(127, std::max(e, m == 0.5 ? k - 1 : k));
        }
    }
    if (e > kQExpMax) return false;
    const double sc = std::ldexp(1.0, e);
    z.scale = (float)sc;                             // exact: a normal power of two
    for (int a = 0; a < 3; a++) {
        auto empty = [&](int i) { return n.link[i] == kEmpty || !(n.lo[a][i] <= n.hi[a][i]); };
        for (int w = 0; w < 6; w++) z.ax[a][w] = 0;
        for (int i = 0; i < 4; i++) {
            uint32_t l = kHalfHMax, h = 0;           // empty slot: inverted box
            if (!empty(i)) {
                // exact in double: float differences, power-of-two scale
                l = half_round(std::min(kHMax, ((double)n.lo[a][i] - lo[a]) / sc), false);
                h = half_round(std::min(kHMax, ((double)n.hi[a][i] - lo[a]) / sc), true);
            }
            z.ax[a][i / 2] |= l << (16 * (i % 2));
            z.ax[a][2 + i / 2] |= h << (16 * (i % 2));
        }
        z.ax[a][4] = z.ax[a][0];
        z.ax[a][5] = z.ax[a][1];
    }
    return true;
}

// Returns false if a child box is not finite (NaN/inf geometry) or a node is
// too large for kQExpMax: the caller then uses the brute-force scan.  Nodes
// are independent: `threads` host threads share them.
inline bool quantize(const Result4 &Q, std::vector<Node4H> &out, int threads = 1) {
    out.assign(Q.nodes.size(), Node4H{});
    std::atomic<bool> ok{true};
    parallel_ranges(Q.nodes.size(), threads, [&](size_t b, size_t e) {
        for (size_t k = b; k < e; k++)
            if (!quantize_node(Q.nodes[k], out[k])) ok.store(false);
    });
    return ok.load();
}
// The device node format: Node4H (104 B, binary16 planes with octant
// windows).  Round 5 measured a 64-B node with 8-bit planes against it in one
// GPU run, interleaved (profiles/r05/ab_node8_*.txt): C3 -4.1 %, C4 -6.3 %, C5
// -3.2 % -- one 16-B load fewer per node visit does not pay for the 18 VALU
// instructions of its decode nor for the 0.7-1 % more box tests of the
// coarser planes; removed in round 6 (git history keeps it).
using NodeDev = Node4H;
constexpr int kNodeDevLinkOff = kNodeLinkOff;

// Renumber Q's nodes breadth-first (root stays 0), so that the top levels of
// the tree are nodes [0, K) for any K.
template <int W>
inline void bfs_order(ResultW<W> &Q) {
    if (Q.nodes.empty()) return;
    std::vector<int32_t> order;          // new -> old
    std::vector<int32_t> remap(Q.nodes.size(), -1);
    order.push_back(0);
    remap[0] = 0;
    for (size_t h = 0; h < order.size(); h++) {
        const NodeW<W> &n = Q.nodes[order[h]];
        for (int i = 0; i < W; i++) {
            int32_t l = n.link[i];
            if (l >= 0 && remap[l] < 0) {
                remap[l] = (int32_t)order.size();
                order.push_back(l);
            }
        }
    }
    std::vector<NodeW<W>> out(order.size());
    for (size_t k = 0; k < order.size(); k++) {
        out[k] = Q.nodes[order[k]];
        for (int i = 0; i < W; i++)
            if (out[k].link[i] >= 0) out[k].link[i] = remap[out[k].link[i]];
    }
    Q.nodes.swap(out);
}

// Leaf record stream: the device reads a leaf's primitives from one
// contiguous run of 16-B words (no key indirection, one batch of loads per
// primitive).  Rewrites every leaf link of Q (encoded against `keys` as
// leaf_link) to
//     -(1 + (off << 8 | nfaces << 4 | count)),   off in 16-B words, < 2^23
// with the leaf's faces first, then its spheres (each group in key order).
// is_face(key) tells the kind; emit(key) appends the primitive's words and
// returns how many it appended.  Returns false if `off` outgrows its field.
inline void leaf_decode(int32_t link, int &off, int &nfaces, int &count) {
    int v = -link - 1;
    off = v >> 8;
    nfaces = (v >> 4) & 15;
    count = v & 15;
}
template <int W, class IsFace, class Emit>
inline bool leaf_records(ResultW<W> &Q, const std::vector<int32_t> &keys, IsFace is_face, Emit emit,
                         size_t base_words = 0) {
    size_t words = base_words;            // the stream may already hold other trees' records
    for (NodeW<W> &n : Q.nodes) {
        for (int i = 0; i < W; i++) {
            int32_t l = n.link[i];
            if (l >= 0 || l == kEmpty) continue;
            int v = -l - 1, first = v >> 4, count = v & 15;
            // faces first, each kind in key order (a stable insertion sort:
            // count <= 15)
            // (a primitive with several references in the leaf -- build_accel's
            // presplit -- is recorded once)
            int32_t ks[16];
            bool fs[16];
            int m = 0;
            for (int q = 0; q < count; q++) {
                const int32_t k = keys[(size_t)first + q];
                if (std::find(ks, ks + m, k) != ks + m) continue;
                const bool f = is_face(k);
                int w = m++;
                while (w > 0 && (fs[w - 1] != f ? f : k < ks[w - 1])) ks[w] = ks[w - 1], fs[w] = fs[w - 1], w--;
                ks[w] = k, fs[w] = f;
            }
            count = m;
            int nfaces = 0;
            for (int q = 0; q < count; q++) nfaces += fs[q] ? 1 : 0;
            // off <= 2^23 - 2 keeps every link above INT_MIN + 256 (device sentinels)
            if (words >= (size_t(1) << 23) - 1) return false;
            n.link[i] = -(1 + (int32_t)((words << 8) | (size_t)(nfaces << 4) | (size_t)count));
            for (int q = 0; q < count; q++) words += (size_t)emit(ks[q]);
        }
    }
    return true;
}

// Binned SAH builder of the binary tree.  Nodes are numbered depth-first
// (a node, then its left subtree, then its right subtree: children have larger
// indices than their parent, which collapse_sah relies on).  The builder
// reorders the primitive array itself (sequential passes over each range,
// not an index indirection), in the order an index permutation would take.
// With threads > 1 large subtrees are built on their own threads into their
// own node arrays and spliced back in that order: the tree is the same for
// every thread count (tests/test_bvh_host.py checks it bit for bit).
class Builder {
   public:
#ifndef RT_SAH_BINS
#define RT_SAH_BINS 64  // 32 -> 64: box tests -1.2 %, C3 +0.4 % (A/B)
#endif
    static constexpr int kBins = RT_SAH_BINS;
    int max_leaf = 8;                       // SAH leaves (<= 15 fits the link encoding)
    float trav_cost = 1.0f;                 // SAH cost of one node visit, in sphere tests
    int threads = 1;                        // host threads (subtree tasks)
    static constexpr int kSahDepth = 22;    // deeper: object-median splits (bounded depth)
    static constexpr int kMaxDepth = 64;    // binary depth cap (object-median splits below kSahDepth keep it low)
    static constexpr int kForkMin = 2048;   // smallest subtree built on a thread of its own

    // prims: reordered by the build (leaf order)
    explicit Builder(std::vector<Prim> &prims) : P(prims) {}

    // Returns false if the tree would be deeper than kMaxDepth.
    bool build(Result &R) {
        R = Result();
        if (P.empty()) return true;
        const int n = (int)P.size();
        forks.store(std::max(0, threads - 1));
        Sub S;
        S.nodes.reserve(P.size());
        S.nodes.emplace_back();                       // the root is node 0
        Range all = range(0, n);
        int mid = split_point(0, n, 1, all);
        if (mid < 0) mid = n;                         // everything in one leaf
        const Range lr = range(0, mid), rr = range(mid, n);
        int32_t l = leaf_link(0, 0), r = leaf_link(0, 0);
        children(0, mid, n, 2, lr, rr, l, r, S, mid > 0, mid < n);
        set_child(S.nodes[0], 0, lr.box, l);
        set_child(S.nodes[0], 1, rr.box, r);
        R.nodes.swap(S.nodes);
        R.depth = std::max(S.depth, 1);
        R.keys.resize(P.size());
        R.costs.resize(P.size());
        for (size_t i = 0; i < P.size(); i++) R.keys[i] = P[i].key, R.costs[i] = P[i].cost;
        return R.depth <= kMaxDepth;
    }

   private:
    std::vector<Prim> &P;
    std::atomic<int> forks{0};              // threads still free for subtrees

    struct Sub {                            // a subtree's nodes, numbered from 0
        std::vector<Node> nodes;
        int depth = 0;
    };
    struct Range {                          // a range's bounds, centroid bounds and cost
        Box box, cbox;
        float cost = 0.0f;                  // summed in array order
    };

    Range range(int a, int b) const {
        Range r;
        for (int i = a; i < b; i++) {
            r.box.grow(P[i].box);
            r.cbox.grow(P[i].c);
            r.cost += P[i].cost;
        }
        return r;
    }

    static void set_child(Node &n, int side, const Box &b, int32_t link) {
        if (side == 0) {
            n.l_lo[0] = b.lo[0], n.l_lo[1] = b.lo[1], n.l_lo[2] = b.lo[2];
            n.l_hi0 = b.hi[0], n.l_hi12[0] = b.hi[1], n.l_hi12[1] = b.hi[2];
        } else {
            n.r_lo01[0] = b.lo[0], n.r_lo01[1] = b.lo[1], n.r_lo2 = b.lo[2];
            n.r_hi[0] = b.hi[0], n.r_hi[1] = b.hi[1], n.r_hi[2] = b.hi[2];
        }
        n.link[side] = link;
    }

    // The best binned split of one axis, in the order a dense sweep over
    // every bin visits it (k from kBins - 1 down, strict '<'): updates (best,
    // best_axis, best_bin).  bins[0..m) are the non-empty bins, ascending
    // (dense: m = kBins, bins = 0..kBins-1).  Every k in (bins[j-1], bins[j]]
    // splits the same sets at the same cost and the dense sweep meets
    // k = bins[j] first; empty bins add +0 to the cost sums (exact), so both
    // forms choose the same split.
    static void sweep(const Box *bb, const float *cc, const int *bins, int m, int ax, float &best, int &best_axis,
                      int &best_bin) {
        // left areas only (the boxes themselves are not needed after it);
        // no default-constructed box arrays: this runs once per axis for
        // every node of a tree built down to single primitives
        float la[kBins];
        float lc[kBins];
        Box acc;
        float c = 0;
        for (int j = 0; j < m; j++) {
            acc.grow(bb[j]);
            c += cc[j];
            la[j] = acc.area();
            lc[j] = c;
        }
        acc = Box();
        c = 0;
        for (int j = m - 1; j > 0; j--) {
            acc.grow(bb[j]);
            c += cc[j];
            if (lc[j - 1] == 0 || c == 0) continue;
            float s = la[j - 1] * lc[j - 1] + acc.area() * c;
            if (s < best) best = s, best_axis = ax, best_bin = bins[j];
        }
    }

    // kBins boxes, not constructed (filled before they are read)
    struct BoxStore {
        union {
            Box b[kBins];
        };
        BoxStore() {}
    };

    static int bin_of(const Prim &p, int ax, float lo, float scale) {
        return std::min(kBins - 1, std::max(0, (int)((p.c[ax] - lo) * scale)));
    }

    // Partition [a, b) (its Range ri) and return the split position, or -1
    // for "make a leaf".
    int split_point(int a, int b, int depth, const Range &ri) {
        int n = b - a;
        if (n <= 1) return -1;
        const Box &cb = ri.cbox;
        const float cost_leaf = ri.cost;
        if (depth > kSahDepth) {
            if (n <= 2) return -1;
            int ax = 0;
            for (int k = 1; k < 3; k++)
                if (cb.hi[k] - cb.lo[k] > cb.hi[ax] - cb.lo[ax]) ax = k;
            int mid = a + n / 2;
            std::nth_element(P.begin() + a, P.begin() + mid, P.begin() + b,
                             [&](const Prim &x, const Prim &y) { return x.c[ax] < y.c[ax]; });
            return mid;
        }
        float best = INFINITY;
        int best_axis = -1, best_bin = -1;
        float lo[3], scale[3];
        bool live[3];
        for (int ax = 0; ax < 3; ax++) {
            lo[ax] = cb.lo[ax];
            live[ax] = cb.hi[ax] > lo[ax];
            scale[ax] = live[ax] ? kBins / (cb.hi[ax] - lo[ax]) : 0.0f;
        }
        if (n < kBins / 2) {
            // few primitives: only their bins, sorted per axis
            for (int ax = 0; ax < 3; ax++) {
                if (!live[ax]) continue;
                BoxStore bb;
                float cc[kBins];
                int bins[kBins];
                int key[kBins];
                int m = 0;
                for (int i = 0; i < n; i++) key[i] = (bin_of(P[a + i], ax, lo[ax], scale[ax]) << 8) | i;
                std::sort(key, key + n);
                for (int t = 0; t < n; t++) {
                    const int k = key[t] >> 8;
                    const Prim &p = P[a + (key[t] & 255)];
                    if (m == 0 || bins[m - 1] != k) bins[m] = k, bb.b[m] = Box(), cc[m] = 0.0f, m++;
                    bb.b[m - 1].grow(p.box);
                    cc[m - 1] += p.cost;
                }
                sweep(bb.b, cc, bins, m, ax, best, best_axis, best_bin);
            }
        } else {
            // one pass over the range bins all three axes
            Box bb[3][kBins];
            float cc[3][kBins];
            int bins[kBins];
            for (int k = 0; k < kBins; k++) cc[0][k] = cc[1][k] = cc[2][k] = 0.0f, bins[k] = k;
            for (int i = a; i < b; i++) {
                const Prim &p = P[i];
                for (int ax = 0; ax < 3; ax++) {
                    const int k = bin_of(p, ax, lo[ax], scale[ax]);
                    bb[ax][k].grow(p.box);
                    cc[ax][k] += p.cost;
                }
            }
            for (int ax = 0; ax < 3; ax++)
                if (live[ax]) sweep(bb[ax], cc[ax], bins, kBins, ax, best, best_axis, best_bin);
        }
        float area = ri.box.area();
        float split_cost = (best_axis >= 0 && area > 0) ? trav_cost + best / area : INFINITY;
        if (n <= max_leaf && split_cost >= cost_leaf) return -1;
        if (best_axis < 0) {                         // all centroids coincide
            if (n <= 15) return -1;
            return a + n / 2;
        }
        const float blo = lo[best_axis], bsc = scale[best_axis];
        auto it = std::partition(P.begin() + a, P.begin() + b,
                                 [&](const Prim &p) { return bin_of(p, best_axis, blo, bsc) < best_bin; });
        int mid = (int)(it - P.begin());
        if (mid == a || mid == b) mid = a + n / 2;
        return mid;
    }

    // The two children of a node over [a, mid) and [mid, b): on this thread,
    // or the left one on a thread of its own when the range is large
    void children(int a, int mid, int b, int depth, const Range &lr, const Range &rr, int32_t &l, int32_t &r,
                  Sub &out, bool has_l = true, bool has_r = true) {
        if (has_l && has_r && b - a >= kForkMin && forks.fetch_sub(1) > 0) {
            Sub L, Rs;
            std::thread t([&] { l = build_range(a, mid, depth, lr, L); });
            r = build_range(mid, b, depth, rr, Rs);
            t.join();
            const int offL = (int)out.nodes.size(), offR = offL + (int)L.nodes.size();
            auto splice = [&](Sub &S, int off) {
                for (Node nd : S.nodes) {
                    for (int k = 0; k < 2; k++)
                        if (nd.link[k] >= 0) nd.link[k] += off;
                    out.nodes.push_back(nd);
                }
                out.depth = std::max(out.depth, S.depth);
            };
            splice(L, offL);
            splice(Rs, offR);
            if (l >= 0) l += offL;
            if (r >= 0) r += offR;
            return;
        }
        if (has_l) l = build_range(a, mid, depth, lr, out);
        if (has_r) r = build_range(mid, b, depth, rr, out);
    }

    int32_t build_range(int a, int b, int depth, const Range &ri, Sub &out) {
        out.depth = std::max(out.depth, depth);
        int mid = split_point(a, b, depth, ri);
        if (mid < 0) return leaf_link(a, b - a);
        int ni = (int)out.nodes.size();
        out.nodes.emplace_back();
        const Range lr = range(a, mid), rr = range(mid, b);
        int32_t l, r;
        children(a, mid, b, depth + 1, lr, rr, l, r, out);
        set_child(out.nodes[ni], 0, lr.box, l);
        set_child(out.nodes[ni], 1, rr.box, r);
        return ni;
    }
};

}  // namespace rtbvh
