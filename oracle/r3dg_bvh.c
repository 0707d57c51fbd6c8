/*
 * r3dg_bvh.c -- CPU restatement of the reference's BVH visibility tracer.
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ (and nothing in the product) as the checker of
 * relightable3dgaussian_amd/csrc/bvh.hip.
 *
 * Follows, operation for operation (compiled with -ffp-contract=off, see Makefile):
 *   oracle_bvh_leaf_aabbs   bvh/__init__.py:29-59 (RayTracer.__init__ corner boxes) with
 *                           utils/general_utils.py:82-103 (build_rotation)
 *   oracle_bvh_build        bvh/src/construct.cu:148-265 (bounds reduce, Morton codes :22-53,
 *                           stable sort, 61-bit keys, determine_range :55-115, find_split
 *                           :117-146, bottom-up boxes and counts :231-264)
 *   oracle_bvh_trace_opacity bvh/src/trace.cu:199-286 with utility.cuh:35-113
 *   oracle_bvh_trace         bvh/src/trace.cu:8-196 (count pass, emission pass, stable sort)
 *
 * Pinning: the leaf boxes are pinned by tests/golden/bvh.npz, produced by running the
 * reference's own RayTracer.__init__ torch code on CPU (tests/golden/make_golden_bvh.py).
 * The tree build and the traces are CUDA-only in the reference (no nvcc / GPU here, no tests or
 * fixtures upstream): parity for them is pinned by this restatement alone, plus structural
 * properties checked in tests/test_bvh.py (a valid binary tree over all leaves, subtree counts,
 * parent boxes enclosing child boxes, ray results against brute force over all Gaussians).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float lx, ly, lz, ux, uy, uz;
} box_t;

static box_t ld_box(const float* a, long i) {
    box_t b;
    memcpy(&b, a + 6 * i, sizeof b);
    return b;
}
static void st_box(float* a, long i, box_t b) { memcpy(a + 6 * i, &b, sizeof b); }

static box_t merge(box_t a, box_t b) {
    box_t m = {fminf(a.lx, b.lx), fminf(a.ly, b.ly), fminf(a.lz, b.lz),
               fmaxf(a.ux, b.ux), fmaxf(a.uy, b.uy), fmaxf(a.uz, b.uz)};
    return m;
}

void oracle_bvh_leaf_aabbs(int P, const float* means, const float* scales, const float* rots, float* out) {
    for (int i = 0; i < P; ++i) {
        const float* q = rots + 4 * (long)i;
        const float norm = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        const float r = q[0] / norm, x = q[1] / norm, y = q[2] / norm, z = q[3] / norm;
        float R[3][3];
        R[0][0] = 1 - 2 * (y * y + z * z);
        R[0][1] = 2 * (x * y - r * z);
        R[0][2] = 2 * (x * z + r * y);
        R[1][0] = 2 * (x * y + r * z);
        R[1][1] = 1 - 2 * (x * x + z * z);
        R[1][2] = 2 * (y * z - r * x);
        R[2][0] = 2 * (x * z - r * y);
        R[2][1] = 2 * (y * z + r * x);
        R[2][2] = 1 - 2 * (x * x + y * y);
        const float sa = 3 * scales[3 * (long)i], sb = 3 * scales[3 * (long)i + 1], sc = 3 * scales[3 * (long)i + 2];
        for (int k = 0; k < 3; ++k) {
            const float m = means[3 * (long)i + k];
            const float as = R[k][0] * sa, bs = R[k][1] * sb, cs = R[k][2] * sc;
            /* x111, x110, x101, x100, x011, x010, x001, x000 of bvh/__init__.py:45-52 */
            const float v[8] = {m + as + bs + cs, m + as + bs - cs, m + as - bs + cs, m + as - bs - cs,
                                m - as + bs + cs, m - as + bs - cs, m - as - bs + cs, m - as - bs - cs};
            float lo = v[0], hi = v[0];
            for (int j = 1; j < 8; ++j) {
                lo = fminf(lo, v[j]);
                hi = fmaxf(hi, v[j]);
            }
            out[6 * (long)i + k] = lo;
            out[6 * (long)i + 3 + k] = hi;
        }
    }
}

static uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

static uint32_t morton_of(box_t b, box_t w) {
    float p[3] = {(float)((double)(b.ux + b.lx) * 0.5), (float)((double)(b.uy + b.ly) * 0.5),
                  (float)((double)(b.uz + b.lz) * 0.5)};
    const float lo[3] = {w.lx, w.ly, w.lz}, hi[3] = {w.ux, w.uy, w.uz};
    uint32_t e[3];
    for (int k = 0; k < 3; ++k) {
        p[k] -= lo[k];
        p[k] /= (hi[k] - lo[k]);
        p[k] = fminf(fmaxf(p[k] * 1024.0f, 0.0f), 1024.0f - 1.0f);
        e[k] = expand_bits((uint32_t)p[k]);
    }
    return e[0] * 4 + e[1] * 2 + e[2];
}

typedef struct {
    uint32_t code, idx;
} ci_t;

static int ci_cmp(const void* a, const void* b) {
    const ci_t *x = a, *y = b;
    if (x->code != y->code) return x->code < y->code ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);  /* stable: original order breaks ties */
}

static int cub(uint64_t a, uint64_t b) { return a == b ? 64 : __builtin_clzll(a ^ b); }

/* aabbs rows P-1.. hold the leaf boxes in Gaussian order on entry (as the reference's Python
 * fills them); every field of nodes and every row of aabbs is written. Returns 0 or -1. */
int oracle_bvh_build(int P, int32_t* nodes, float* aabbs, uint64_t* keys) {
    if (P < 1) return -1;
    const long ni = P - 1;
    box_t whole = {100000.f, 100000.f, 100000.f, -100000.f, -100000.f, -100000.f};
    for (long i = 0; i < P; ++i) whole = merge(whole, ld_box(aabbs, ni + i));
    ci_t* ci = malloc(sizeof(ci_t) * (size_t)P);
    box_t* leaf = malloc(sizeof(box_t) * (size_t)P);
    if (!ci || !leaf) return -1;
    for (long i = 0; i < P; ++i) {
        leaf[i] = ld_box(aabbs, ni + i);
        ci[i].code = morton_of(leaf[i], whole);
        ci[i].idx = (uint32_t)i;
    }
    qsort(ci, (size_t)P, sizeof(ci_t), ci_cmp);
    for (long i = 0; i < P; ++i) {
        keys[i] = ((uint64_t)ci[i].code << 31) | ci[i].idx;
        st_box(aabbs, ni + i, leaf[ci[i].idx]);
        int32_t* row = nodes + 5 * (ni + i);
        row[0] = -1;
        row[1] = -1;
        row[2] = -1;
        row[3] = (int32_t)ci[i].idx;
        row[4] = 1;
    }
    free(ci);
    free(leaf);
    if (ni > 0) nodes[0] = -1;
    for (int idx = 0; idx < ni; ++idx) {
        int first, last;
        if (idx == 0) {
            first = 0;
            last = P - 1;
        } else {
            const uint64_t self = keys[idx];
            const int dl = cub(self, keys[idx - 1]), dr = cub(self, keys[idx + 1]);
            const int d = dr > dl ? 1 : -1;
            const int dmin = dl < dr ? dl : dr;
            int lmax = 2, delta = -1, it = idx + d * lmax;
            if (0 <= it && it < P) delta = cub(self, keys[it]);
            while (delta > dmin) {
                lmax <<= 1;
                it = idx + d * lmax;
                delta = -1;
                if (0 <= it && it < P) delta = cub(self, keys[it]);
            }
            int l = 0;
            for (int t = lmax >> 1; t > 0; t >>= 1) {
                it = idx + (l + t) * d;
                delta = -1;
                if (0 <= it && it < P) delta = cub(self, keys[it]);
                if (delta > dmin) l += t;
            }
            const int j = idx + l * d;
            first = d < 0 ? j : idx;
            last = d < 0 ? idx : j;
        }
        int gamma;
        if (keys[first] == keys[last]) {
            gamma = (first + last) >> 1;
        } else {
            const int dn = cub(keys[first], keys[last]);
            int split = first, stride = last - first;
            do {
                stride = (stride + 1) >> 1;
                const int middle = split + stride;
                if (middle < last && cub(keys[first], keys[middle]) > dn) split = middle;
            } while (stride > 1);
            gamma = split;
        }
        int lc = gamma, rc = gamma + 1;
        if (first == gamma) lc += (int)ni;
        if (last == gamma + 1) rc += (int)ni;
        int32_t* row = nodes + 5 * (long)idx;
        row[1] = lc;
        row[2] = rc;
        row[3] = -1;
        row[4] = last - first + 1;
        nodes[5 * (long)lc] = idx;
        nodes[5 * (long)rc] = idx;
    }
    /* bottom-up: the second child to arrive merges (left, right) and climbs on */
    char* flag = calloc((size_t)(ni > 0 ? ni : 1), 1);
    if (!flag) return -1;
    for (long i = 0; i < P; ++i) {
        int node = (int)(ni + i);
        int parent = nodes[5 * (long)node];
        while (parent != -1) {
            if (!flag[parent]) {
                flag[parent] = 1;
                break;
            }
            const int l = nodes[5 * (long)parent + 1], r = nodes[5 * (long)parent + 2];
            st_box(aabbs, parent, merge(ld_box(aabbs, l), ld_box(aabbs, r)));
            node = parent;
            parent = nodes[5 * (long)node];
        }
    }
    free(flag);
    return 0;
}

static void ray_box(box_t b, const float* o, const float* d, float* out) {
    float tmin = (b.lx - o[0]) / d[0], tmax = (b.ux - o[0]) / d[0], s;
    if (tmin > tmax) { s = tmin; tmin = tmax; tmax = s; }
    float tymin = (b.ly - o[1]) / d[1], tymax = (b.uy - o[1]) / d[1];
    if (tymin > tymax) { s = tymin; tymin = tymax; tymax = s; }
    if (tmin > tymax || tymin > tmax) { out[0] = out[1] = -1.f; return; }
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (b.lz - o[2]) / d[2], tzmax = (b.uz - o[2]) / d[2];
    if (tzmin > tzmax) { s = tzmin; tzmin = tzmax; tzmax = s; }
    if (tmin > tzmax || tzmin > tmax) { out[0] = out[1] = -1.f; return; }
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    out[0] = tmin;
    out[1] = tmax;
}

/* the child with the larger exit distance is pushed first; exits <= 0 are dropped */
static int push_children(const int32_t* nodes, const float* aabbs, int node, const float* o, const float* d,
                         int* ids, float* spans) {
    const int l = nodes[5 * (long)node + 1], r = nodes[5 * (long)node + 2];
    float il[2], ir[2];
    ray_box(ld_box(aabbs, l), o, d, il);
    ray_box(ld_box(aabbs, r), o, d, ir);
    int n = 0;
#define PUSH(id, iv)                                        \
    do {                                                    \
        ids[n] = id;                                        \
        if (spans) { spans[2 * n] = iv[0]; spans[2 * n + 1] = iv[1]; } \
        ++n;                                                \
    } while (0)
    if (il[1] > ir[1]) {
        if (il[1] > 0) PUSH(l, il);
        if (ir[1] > 0) PUSH(r, ir);
    } else {
        if (ir[1] > 0) PUSH(r, ir);
        if (il[1] > 0) PUSH(l, il);
    }
#undef PUSH
    return n;
}

#define STACK 128

/* t_last (optional): the transmittance after the last contributing Gaussian (before the 0.9
 * cut), so tests can tell rays that sit on the threshold */
void oracle_bvh_trace_opacity(int R, const int32_t* nodes, const float* aabbs, const float* rays_o,
                              const float* rays_d, const float* means, const float* cov, const float* opac,
                              const float* normals, int32_t* contrib, float* vis, float* t_last, int32_t* nterms) {
    for (int ray = 0; ray < R; ++ray) {
        const float* o = rays_o + 3 * (long)ray;
        const float* d = rays_d + 3 * (long)ray;
        int stack[STACK], sp = 0, count = 0, done = 0;
        stack[sp++] = 0;
        float T = 1.f;
        while (sp > 0 && !done) {
            const int node = stack[--sp];
            const int32_t* row = nodes + 5 * (long)node;
            if (row[4] <= 1) {
                const int g = row[3];
                if (opac[g] < 1.f / 255.f) continue;
                const float* n = normals + 3 * (long)g;
                if (n[0] * d[0] + n[1] * d[1] + n[2] * d[2] > 0) continue;
                const float* m = means + 3 * (long)g;
                const float* c = cov + 6 * (long)g;
                const float mx = m[0] - o[0], my = m[1] - o[1], mz = m[2] - o[2];
                const float t1 = c[0] * mx * d[0] + c[1] * mx * d[1] + c[2] * mx * d[2] + c[1] * my * d[0] +
                                 c[3] * my * d[1] + c[4] * my * d[2] + c[2] * mz * d[0] + c[4] * mz * d[1] +
                                 c[5] * mz * d[2];
                const float t2 = c[0] * d[0] * d[0] + c[1] * d[0] * d[1] + c[2] * d[0] * d[2] + c[1] * d[1] * d[0] +
                                 c[3] * d[1] * d[1] + c[4] * d[1] * d[2] + c[2] * d[2] * d[0] + c[4] * d[2] * d[1] +
                                 c[5] * d[2] * d[2];
                const float t = t1 / t2;
                if (t < 0.01) continue;
                const float p[3] = {o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]};
                const float dx = m[0] - p[0], dy = m[1] - p[1], dz = m[2] - p[2];
                const float power = (float)(-0.5 * (dx * dx * c[0] + dy * dy * c[3] + dz * dz * c[5] +
                                                     2 * dx * dy * c[1] + 2 * dx * dz * c[2] + 2 * dy * dz * c[4]));
                if (power > 0) continue;
                count += 1;
                const float alpha = opac[g] * expf(power);
                T *= 1 - alpha;
                if (T < 0.9) done = 1;
            } else {
                int ids[2];
                const int n = push_children(nodes, aabbs, node, o, d, ids, NULL);
                for (int k = 0; k < n; ++k) stack[sp++] = ids[k];
            }
        }
        if (t_last) t_last[ray] = T;
        if (nterms) nterms[ray] = count; /* factors multiplied into T, up to and including the cut */
        contrib[ray] = done ? 0 : count;
        vis[ray] = done ? 0.f : T;
    }
}

typedef struct {
    uint32_t tbits;
    int32_t point;
    float pos[3];
} rec_t;

/* pass 1 when point == NULL: per-ray counts into contrib, returns L. pass 2: fills the lists
 * (point [L], position [L, 3], ray_id [L]) sorted by (ray, t), stable. */
long oracle_bvh_trace(int R, const int32_t* nodes, const float* aabbs, const float* rays_o, const float* rays_d,
                      const float* means, int32_t* contrib, int32_t* point, float* position, int32_t* ray_id) {
    long L = 0;
    for (int ray = 0; ray < R; ++ray) {
        const float* o = rays_o + 3 * (long)ray;
        const float* d = rays_d + 3 * (long)ray;
        int stack[STACK], sp = 0;
        float span[2 * STACK];
        stack[sp] = 0;
        span[0] = -1000.f;
        span[1] = 1000.f;
        ++sp;
        const long base = L;
        while (sp > 0) {
            --sp;
            const int node = stack[sp];
            const float in0 = span[2 * sp], in1 = span[2 * sp + 1];
            const int32_t* row = nodes + 5 * (long)node;
            if (row[4] <= 4) {
                if (!point) {
                    L += row[4];
                    continue;
                }
                int st2[8], sp2 = 0;
                st2[sp2++] = node;
                while (sp2 > 0) {
                    const int n2 = st2[--sp2];
                    const int32_t* r2 = nodes + 5 * (long)n2;
                    if (r2[3] >= 0) {
                        int g = r2[3];
                        const float* m = means + 3 * (long)g;
                        float t = (m[0] - o[0]) * d[0] + (m[1] - o[1]) * d[1] + (m[2] - o[2]) * d[2];
                        if (t < 0.01 || t < in0 || t > in1) {
                            t = 1000000.f;
                            g = -1;
                        }
                        point[L] = g;
                        ray_id[L] = ray;
                        position[3 * L] = o[0] + t * d[0];
                        position[3 * L + 1] = o[1] + t * d[1];
                        position[3 * L + 2] = o[2] + t * d[2];
                        ++L;
                    } else {
                        st2[sp2++] = r2[1];
                        st2[sp2++] = r2[2];
                    }
                }
            } else {
                int ids[2];
                float sp_[4];
                const int n = push_children(nodes, aabbs, node, o, d, ids, sp_);
                for (int k = 0; k < n; ++k) {
                    stack[sp] = ids[k];
                    span[2 * sp] = sp_[2 * k];
                    span[2 * sp + 1] = sp_[2 * k + 1];
                    ++sp;
                }
            }
        }
        if (!point) {
            contrib[ray] = (int32_t)(L - base);
            continue;
        }
        /* stable insertion sort of this ray's records by bits(t); t is recovered exactly from
         * the stored record (rejected: 1e6) by recomputing it in the same order */
        const long n = L - base;
        rec_t* rec = malloc(sizeof(rec_t) * (size_t)(n > 0 ? n : 1));
        for (long k = 0; k < n; ++k) {
            const long s = base + k;
            rec[k].point = point[s];
            memcpy(rec[k].pos, position + 3 * s, sizeof rec[k].pos);
            float t;
            if (point[s] < 0) {
                t = 1000000.f;
            } else {
                const float* m = means + 3 * (long)point[s];
                t = (m[0] - o[0]) * d[0] + (m[1] - o[1]) * d[1] + (m[2] - o[2]) * d[2];
            }
            memcpy(&rec[k].tbits, &t, 4);
        }
        for (long k = 1; k < n; ++k) {
            rec_t x = rec[k];
            long j = k - 1;
            while (j >= 0 && rec[j].tbits > x.tbits) {
                rec[j + 1] = rec[j];
                --j;
            }
            rec[j + 1] = x;
        }
        for (long k = 0; k < n; ++k) {
            point[base + k] = rec[k].point;
            memcpy(position + 3 * (base + k), rec[k].pos, sizeof rec[k].pos);
        }
        free(rec);
    }
    return L;
}
