/*
 * oracle/rt_oracle.c -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product path (rf_ray_tracing_warp_amd) never links or calls it.
 *
 * What it restates (reference = /root/reference, rmenon1008/rf_ray_tracing_warp):
 *   kernel.py:38-98   trace_paths_kernel  (one ray per loop iteration, B bounces)
 *   kernel.py:6-8     reflect
 *   kernel.py:51-52   wp.rand_init / wp.sample_unit_sphere_surface   (warp-lang, not vendored)
 *   kernel.py:71,82   wp.mesh_query_ray  closest hit                  (warp-lang, not vendored)
 *
 * Pinning status (see DESIGN.md "Oracle"):
 *   - ray generation (PCG + sphere sampling): PINNED -- the 119 received paths stored in the
 *     reference's own artifact web/scene.html start in directions this restatement generates
 *     for 119 ray ids to <= 2.6e-8 rad (tests/golden/scene_html.npz).
 *   - RX icosphere geometry: PINNED bit-exactly (f32) by the same artifact.
 *   - triangle test / closest hit: restates warp-lang's mesh_query_ray + watertight ray/triangle
 *     test (Woop, Benthin & Wald 2013) with the fused multiply-adds nvcc's LLVM contraction
 *     produces.  PINNED by the artifact: 117/119 first hit points are bit-identical to the
 *     reference's f32 output and 118/119 path structures match (test_golden_scene_html).
 *     Env-reflection arithmetic (dot, normalize, reflect) follows the same contraction rule but
 *     the artifact has no env bounce, so that part is pinned only by the rule, not by data.
 *   - tie between two triangles at exactly equal t: Warp keeps the first found in BVH order;
 *     this restatement takes the lowest face id (order independent).  "Parity unpinned" there.
 *
 * Arithmetic contract (shared, by restatement, with the HIP kernels in
 * rf_ray_tracing_warp_amd/csrc/rt_device.h -- written independently, they must agree bit for
 * bit; compile with -ffp-contract=off and no fast-math so only the explicit fmaf fuse):
 *   dot(a,b)     = fmaf(a.z,b.z, fmaf(a.x,b.x, a.y*b.y))       [a.x*b.x + a.y*b.y + a.z*b.z]
 *   cross(a,b)   = (fmaf(a.y,b.z,-(a.z*b.y)), fmaf(a.z,b.x,-(a.x*b.z)), fmaf(a.x,b.y,-(a.y*b.x)))
 *   normalize(v) = v/l per component, l = sqrtf(dot(v,v)); 0 vector if l == 0
 *   face normal  = normalize(cross(q-p, r-p)), corners in index order
 *   watertight test (see orc_tri_test): kz = longest |dir| axis, shear S = dir[k]/dir[kz],
 *       A = a-o ...; Ax = fmaf(-Sx, A[kz], A[kx]) ...; U = fmaf(Cx,By,-(Cy*Bx)) ...;
 *       zero U/V/W recomputed in double; T = fmaf(W,Cz, fmaf(U,Az, V*Bz)); t = T*(1.0f/det)
 *   closest hit  = lexicographic min of (t, face) over hits with 0 <= t < max_t
 *   advance      p' = fmaf(d, t, p) per component                       (kernel.py:87,94)
 *   reflect      s = 2*dot(d,n);  d' = fmaf(-s, n, d)  (no renormalisation, kernel.py:6-8)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define RT_MAX_T 1.0e6f /* kernel.py:71,82 */

/* ---------------- ray generation (kernel.py:51-52, warp rand.h semantics) --------------- */
uint32_t orc_pcg(uint32_t s)
{
    uint32_t b = s * 747796405u + 2891336453u;
    uint32_t c = ((b >> ((b >> 28u) + 4u)) ^ b) * 277803737u;
    return (c >> 22u) ^ c;
}

static float orc_randf(uint32_t* st)
{
    *st = orc_pcg(*st);
    return (float)(*st >> 8) * (1.0f / 16777216.0f);
}

/* f32 sin/cos on a Cody-Waite reduced argument; fixed polynomials (Cephes-style
 * minimax coefficients), evaluated with explicit fmaf so CPU and GPU agree. */
static float sin_poly(float r)
{
    float z = r * r;
    float p = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(z, p, -1.6666654611e-1f);
    return fmaf(r * z, p, r);
}
static float cos_poly(float r)
{
    float z = r * r;
    float p = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(z, p, 4.166664568298827e-2f);
    return fmaf(z * z, p, fmaf(-0.5f, z, 1.0f));
}
#define PIO2_HI 1.57079637050628662109375f       /* f32(pi/2) */
#define PIO2_LO -4.37113900018624283e-8f         /* pi/2 - PIO2_HI */
#define TWO_OVER_PI 0.636619746685028076171875f  /* f32(2/pi) */
void orc_sincosf(float x, float* s, float* c)
{
    float k = rintf(x * TWO_OVER_PI);
    float r = fmaf(-k, PIO2_HI, x);
    r = fmaf(-k, PIO2_LO, r);
    float sp = sin_poly(r), cp = cos_poly(r);
    int q = ((int)k) & 3;
    switch (q) {
    case 0: *s = sp; *c = cp; break;
    case 1: *s = cp; *c = -sp; break;
    case 2: *s = -sp; *c = -cp; break;
    default: *s = -cp; *c = sp; break;
    }
}
static float asin_small(float x) /* |x| <= 0.5 */
{
    float z = x * x;
    float p = fmaf(4.2163199048e-2f, z, 2.4181311049e-2f);
    p = fmaf(p, z, 4.5470025998e-2f);
    p = fmaf(p, z, 7.4953002686e-2f);
    p = fmaf(p, z, 1.6666752422e-1f);
    return fmaf(p * z, x, x);
}
#define PI_F 3.14159274101257324219f
float orc_acosf(float x)
{
    if (x < -0.5f) return PI_F - 2.0f * asin_small(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asin_small(sqrtf(0.5f * (1.0f - x)));
    return PIO2_HI - asin_small(x);
}

/* wp.sample_unit_sphere_surface(wp.rand_init(tid))  (kernel.py:51-52) */
void orc_ray_dir(int64_t gid, float d[3])
{
    uint32_t st = orc_pcg((uint32_t)gid);
    float u1 = orc_randf(&st);
    float phi = orc_acosf(1.0f - 2.0f * u1);
    float u2 = orc_randf(&st);
    float theta = (6.28318548202514648438f - 0.0f) * u2 + 0.0f; /* randf(state, 0, 2*pi) */
    float st_, ct, sp, cp;
    orc_sincosf(theta, &st_, &ct);
    orc_sincosf(phi, &sp, &cp);
    d[0] = ct * sp;
    d[1] = st_ * sp;
    d[2] = cp;
}

/* ---------------- geometry ---------------- */
static inline float dot3(const float* a, const float* b)
{
    return fmaf(a[2], b[2], fmaf(a[0], b[0], a[1] * b[1]));
}
static inline void cross3(const float* a, const float* b, float* o)
{
    o[0] = fmaf(a[1], b[2], -(a[2] * b[1]));
    o[1] = fmaf(a[2], b[0], -(a[0] * b[2]));
    o[2] = fmaf(a[0], b[1], -(a[1] * b[0]));
}

/* prepared mesh: per face the three corners (9 floats) and the unit normal (3 floats); meshes
 * above ORC_BVH_MIN faces also get a simple median-split BVH (double boxes, padded), written
 * independently of the product's SAH BVH -- the closest hit does not depend on the tree. */
static int64_t ORC_BVH_MIN = 2048;
void orc_set_bvh_min(int64_t n) { ORC_BVH_MIN = n; }
#define ORC_LEAF 8
typedef struct {
    double lo[3], hi[3];
    int64_t left, right; /* internal: child node ids; leaf: left = -1, right unused */
    int64_t first, count;
} orc_node;
typedef struct {
    int64_t nf;
    float* tri; /* nf * 12 */
    orc_node* nodes;
    int64_t nnodes;
    int64_t* order; /* leaf-ordered face ids */
} orc_mesh;

static double orc_cen(const orc_mesh* m, int64_t f, int k)
{
    const float* T = m->tri + 12 * f;
    return ((double)T[k] + (double)T[3 + k] + (double)T[6 + k]) / 3.0;
}
static int64_t orc_build(orc_mesh* m, int64_t first, int64_t count, double pad, int64_t* cap)
{
    if (m->nnodes == *cap) {
        *cap *= 2;
        m->nodes = (orc_node*)realloc(m->nodes, sizeof(orc_node) * (size_t)(*cap));
    }
    const int64_t id = m->nnodes++;
    orc_node nd;
    for (int k = 0; k < 3; ++k) {
        nd.lo[k] = INFINITY;
        nd.hi[k] = -INFINITY;
    }
    for (int64_t i = first; i < first + count; ++i) {
        const float* T = m->tri + 12 * m->order[i];
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) {
                if (T[3 * v + k] < nd.lo[k]) nd.lo[k] = T[3 * v + k];
                if (T[3 * v + k] > nd.hi[k]) nd.hi[k] = T[3 * v + k];
            }
    }
    for (int k = 0; k < 3; ++k) {
        nd.lo[k] -= pad;
        nd.hi[k] += pad;
    }
    nd.first = first;
    nd.count = count;
    nd.left = nd.right = -1;
    if (count > ORC_LEAF) {
        int axis = 0;
        double ext = nd.hi[0] - nd.lo[0];
        for (int k = 1; k < 3; ++k)
            if (nd.hi[k] - nd.lo[k] > ext) {
                ext = nd.hi[k] - nd.lo[k];
                axis = k;
            }
        /* median split by centroid: simple insertion-free nth-element via qsort on keys */
        int64_t half = count / 2;
        /* selection by repeated partition (quickselect) on order[first .. first+count) */
        int64_t lo = first, hi = first + count - 1, kth = first + half;
        while (lo < hi) {
            const double pv = orc_cen(m, m->order[(lo + hi) / 2], axis);
            int64_t i = lo, j = hi;
            while (i <= j) {
                while (orc_cen(m, m->order[i], axis) < pv) ++i;
                while (orc_cen(m, m->order[j], axis) > pv) --j;
                if (i <= j) {
                    int64_t t = m->order[i];
                    m->order[i] = m->order[j];
                    m->order[j] = t;
                    ++i;
                    --j;
                }
            }
            if (kth <= j) hi = j;
            else if (kth >= i) lo = i;
            else break;
        }
        const int64_t l = orc_build(m, first, half, pad, cap);
        const int64_t r = orc_build(m, first + half, count - half, pad, cap);
        nd.left = l;
        nd.right = r;
    }
    m->nodes[id] = nd;
    return id;
}

orc_mesh* orc_mesh_create(const float* verts, int64_t nv, const int32_t* faces, int64_t nf)
{
    (void)nv;
    orc_mesh* m = (orc_mesh*)malloc(sizeof(orc_mesh));
    m->nf = nf;
    m->tri = (float*)malloc(sizeof(float) * 12 * (size_t)(nf > 0 ? nf : 1));
    for (int64_t f = 0; f < nf; ++f) {
        const float* p = verts + 3 * (int64_t)faces[3 * f + 0];
        const float* q = verts + 3 * (int64_t)faces[3 * f + 1];
        const float* r = verts + 3 * (int64_t)faces[3 * f + 2];
        float* T = m->tri + 12 * f;
        memcpy(T, p, 12);
        memcpy(T + 3, q, 12);
        memcpy(T + 6, r, 12);
        float e1[3] = {q[0] - p[0], q[1] - p[1], q[2] - p[2]};
        float e2[3] = {r[0] - p[0], r[1] - p[1], r[2] - p[2]};
        float N[3];
        cross3(e1, e2, N);
        float len = sqrtf(dot3(N, N));
        if (len > 0.0f) {
            T[9] = N[0] / len;
            T[10] = N[1] / len;
            T[11] = N[2] / len;
        } else {
            T[9] = T[10] = T[11] = 0.0f;
        }
    }
    m->nodes = NULL;
    m->nnodes = 0;
    m->order = NULL;
    if (nf > ORC_BVH_MIN) {
        double amax = 0.0;
        for (int64_t i = 0; i < 12 * nf; ++i)
            if (i % 12 < 9 && fabs(m->tri[i]) > amax) amax = fabs(m->tri[i]);
        m->order = (int64_t*)malloc(sizeof(int64_t) * (size_t)nf);
        for (int64_t f = 0; f < nf; ++f) m->order[f] = f;
        int64_t cap = 1024;
        m->nodes = (orc_node*)malloc(sizeof(orc_node) * (size_t)cap);
        orc_build(m, 0, nf, 1e-4 * (1.0 + amax), &cap);
    }
    return m;
}
void orc_mesh_destroy(orc_mesh* m)
{
    if (!m) return;
    free(m->tri);
    free(m->nodes);
    free(m->order);
    free(m);
}

/* per-ray precompute of the watertight test (warp intersect_ray_tri_woop "precompute" block) */
typedef struct {
    int kx, ky, kz;
    float Sx, Sy, Sz;
} orc_shear;

static void orc_shear_init(const float* dir, orc_shear* s)
{
    float ax = fabsf(dir[0]), ay = fabsf(dir[1]), az = fabsf(dir[2]);
    int kz = (ax > ay && ax > az) ? 0 : ((ay > az) ? 1 : 2); /* max_dim / longest_axis */
    int kx = kz + 1;
    if (kx == 3) kx = 0;
    int ky = kx + 1;
    if (ky == 3) ky = 0;
    if (dir[kz] < 0.0f) { /* keep winding */
        int tmp = kx;
        kx = ky;
        ky = tmp;
    }
    s->kx = kx;
    s->ky = ky;
    s->kz = kz;
    s->Sx = dir[kx] / dir[kz];
    s->Sy = dir[ky] / dir[kz];
    s->Sz = 1.0f / dir[kz];
}

/* watertight ray/triangle test; returns 1 and t on hit (t may be >= max_t; caller filters) */
static int orc_tri_test(const float* o, const orc_shear* s, const float* a, const float* b, const float* c,
                        float* t_out)
{
    const int kx = s->kx, ky = s->ky, kz = s->kz;
    float A[3] = {a[0] - o[0], a[1] - o[1], a[2] - o[2]};
    float Bv[3] = {b[0] - o[0], b[1] - o[1], b[2] - o[2]};
    float C[3] = {c[0] - o[0], c[1] - o[1], c[2] - o[2]};
    float Ax = fmaf(-s->Sx, A[kz], A[kx]);
    float Ay = fmaf(-s->Sy, A[kz], A[ky]);
    float Bx = fmaf(-s->Sx, Bv[kz], Bv[kx]);
    float By = fmaf(-s->Sy, Bv[kz], Bv[ky]);
    float Cx = fmaf(-s->Sx, C[kz], C[kx]);
    float Cy = fmaf(-s->Sy, C[kz], C[ky]);
    float U = fmaf(Cx, By, -(Cy * Bx));
    float V = fmaf(Ax, Cy, -(Ay * Cx));
    float W = fmaf(Bx, Ay, -(By * Ax));
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        U = (float)((double)Cx * (double)By - (double)Cy * (double)Bx);
        V = (float)((double)Ax * (double)Cy - (double)Ay * (double)Cx);
        W = (float)((double)Bx * (double)Ay - (double)By * (double)Ax);
    }
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return 0;
    float det = U + V + W;
    if (det == 0.0f) return 0;
    float Az = s->Sz * A[kz];
    float Bz = s->Sz * Bv[kz];
    float Cz = s->Sz * C[kz];
    float T = fmaf(W, Cz, fmaf(U, Az, V * Bz));
    float Ts = (det < 0.0f) ? -T : T; /* xorf(T, sign_mask(det)) */
    if (Ts < 0.0f) return 0;
    float rcp = 1.0f / det;
    *t_out = T * rcp;
    return 1;
}

/* double slab test with slack; returns entry t or INFINITY */
static double orc_slab(const orc_node* nd, const float* o, const float* d)
{
    double tn = 0.0, tf = INFINITY;
    for (int k = 0; k < 3; ++k) {
        if (d[k] == 0.0f) {
            if (o[k] < nd->lo[k] || o[k] > nd->hi[k]) return INFINITY;
            continue;
        }
        double a = (nd->lo[k] - o[k]) / (double)d[k], b = (nd->hi[k] - o[k]) / (double)d[k];
        if (a > b) {
            double t = a;
            a = b;
            b = t;
        }
        if (a > tn) tn = a;
        if (b < tf) tf = b;
    }
    return tn <= tf ? tn : INFINITY;
}

static void orc_consider(const orc_mesh* m, const orc_shear* sh, const float* o, int64_t f, float max_t,
                         float* best_t, int64_t* best_f)
{
    const float* T = m->tri + 12 * f;
    float t;
    if (!orc_tri_test(o, sh, T, T + 3, T + 6, &t)) return;
    if (!(t < max_t && t >= 0.0f)) return;
    if (*best_f < 0 || t < *best_t || (t == *best_t && f < *best_f)) {
        *best_t = t;
        *best_f = f;
    }
}

/* closest hit (mesh_query_ray, kernel.py:71,82): brute force, or the oracle BVH when present */
int orc_query(const orc_mesh* m, const float* o, const float* d, float max_t, float* t_out,
              int32_t* face_out, float* n_out)
{
    orc_shear sh;
    orc_shear_init(d, &sh);
    float best_t = 0.0f;
    int64_t best_f = -1;
    if (m->nodes) {
        int64_t stack[256];
        int sp = 0;
        stack[sp++] = 0;
        while (sp > 0) {
            const orc_node* nd = &m->nodes[stack[--sp]];
            const double te = orc_slab(nd, o, d);
            if (te == INFINITY) continue;
            if (best_f >= 0 && te > (double)best_t * (1.0 + 1e-6) + 1e-6) continue;
            if (nd->left < 0) {
                for (int64_t i = nd->first; i < nd->first + nd->count; ++i)
                    orc_consider(m, &sh, o, m->order[i], max_t, &best_t, &best_f);
            } else {
                stack[sp++] = nd->left;
                stack[sp++] = nd->right;
            }
        }
        if (best_f < 0) return 0;
        *t_out = best_t;
        *face_out = (int32_t)best_f;
        memcpy(n_out, m->tri + 12 * best_f + 9, 12);
        return 1;
    }
    for (int64_t f = 0; f < m->nf; ++f) {
        const float* T = m->tri + 12 * f;
        float t;
        if (!orc_tri_test(o, &sh, T, T + 3, T + 6, &t)) continue;
        if (!(t < max_t && t >= 0.0f)) continue;
        if (best_f < 0 || t < best_t || (t == best_t && f < best_f)) {
            best_t = t;
            best_f = f;
        }
    }
    if (best_f < 0) return 0;
    *t_out = best_t;
    *face_out = (int32_t)best_f;
    memcpy(n_out, m->tri + 12 * best_f + 9, 12);
    return 1;
}

/*
 * trace_paths_kernel restatement (kernel.py:38-98), rays [ray_offset, ray_offset+n), or the
 * explicit ray ids ids[0..n) when ids != NULL.
 * Outputs (row r = ray ray_offset+r), all optional (NULL):
 *   traced   (n, B+1, 3) f32  -- NaN where the reference leaves its host NaN fill
 *   received (n, B+1, 3) f32  -- longest prefix ending at the last RX hit, NaN after
 *   mask     (n,) u32         -- row_mask (kernel.py:91)
 *   hit_kind (n, B) i32       -- per bounce: 0 miss, 1 env, 2 rx   (debug, not in reference)
 *   hit_face (n, B) i32       -- per bounce: face id of the chosen hit, -1 on miss
 */
void orc_trace_ids(const orc_mesh* env, const orc_mesh* rx, const float* tx, int B, int64_t ray_offset,
                   const int64_t* ids, int64_t n, float* traced, float* received, uint32_t* mask,
                   int32_t* hit_kind, int32_t* hit_face, int nthreads)
{
    const int P = B + 1;
    const float qnan = nanf("");
    (void)nthreads;
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t r = 0; r < n; ++r) {
        float path[64][3];
        int last_rx = -1; /* index of last path point written by an RX hit */
        int written = 1;
        float dir[3], pos[3] = {tx[0], tx[1], tx[2]};
        orc_ray_dir(ids ? ids[r] : ray_offset + r, dir);
        memcpy(path[0], pos, 12);
        for (int b = 0; b < B; ++b) {
            float tr = 0, te = 0, nr[3], ne[3];
            int32_t fr = -1, fe = -1;
            int hr = orc_query(rx, pos, dir, RT_MAX_T, &tr, &fr, nr);
            int he = orc_query(env, pos, dir, RT_MAX_T, &te, &fe, ne);
            int kind = 0;
            int32_t face = -1;
            if (hr && (!he || te > tr)) { /* kernel.py:85 */
                for (int k = 0; k < 3; ++k) pos[k] = fmaf(dir[k], tr, pos[k]);
                memcpy(path[b + 1], pos, 12);
                written = b + 2;
                last_rx = b + 1;
                kind = 2;
                face = fr;
            } else if (he) { /* kernel.py:93-96 */
                for (int k = 0; k < 3; ++k) pos[k] = fmaf(dir[k], te, pos[k]);
                memcpy(path[b + 1], pos, 12);
                written = b + 2;
                float s = 2.0f * dot3(dir, ne);
                for (int k = 0; k < 3; ++k) dir[k] = fmaf(-s, ne[k], dir[k]);
                kind = 1;
                face = fe;
            } else {
                /* miss: nothing written; every later iteration repeats this miss */
                for (int bb = b; bb < B; ++bb) {
                    if (hit_kind) hit_kind[r * B + bb] = 0;
                    if (hit_face) hit_face[r * B + bb] = -1;
                }
                break;
            }
            if (hit_kind) hit_kind[r * B + b] = kind;
            if (hit_face) hit_face[r * B + b] = face;
        }
        if (traced) {
            float* row = traced + r * P * 3;
            for (int i = 0; i < P; ++i)
                for (int k = 0; k < 3; ++k) row[3 * i + k] = (i < written) ? path[i][k] : qnan;
        }
        if (received) {
            float* row = received + r * P * 3;
            for (int i = 0; i < P; ++i)
                for (int k = 0; k < 3; ++k) row[3 * i + k] = (i <= last_rx) ? path[i][k] : qnan;
        }
        if (mask) mask[r] = last_rx >= 0 ? 1u : 0u;
    }
}

void orc_trace(const orc_mesh* env, const orc_mesh* rx, const float* tx, int B, int64_t ray_offset,
               int64_t n, float* traced, float* received, uint32_t* mask, int32_t* hit_kind,
               int32_t* hit_face, int nthreads)
{
    orc_trace_ids(env, rx, tx, B, ray_offset, NULL, n, traced, received, mask, hit_kind, hit_face, nthreads);
}

/* bulk helpers for tests */
void orc_ray_dirs(int64_t ray_offset, int64_t n, float* out)
{
    for (int64_t i = 0; i < n; ++i) orc_ray_dir(ray_offset + i, out + 3 * i);
}
void orc_sincosf_bulk(const float* x, int64_t n, float* s, float* c)
{
    for (int64_t i = 0; i < n; ++i) orc_sincosf(x[i], s + i, c + i);
}
void orc_acosf_bulk(const float* x, int64_t n, float* out)
{
    for (int64_t i = 0; i < n; ++i) out[i] = orc_acosf(x[i]);
}
int orc_query_bulk(const orc_mesh* m, const float* o, const float* d, int64_t n, float max_t,
                   float* t, int32_t* face, float* nrm)
{
    int hits = 0;
    for (int64_t i = 0; i < n; ++i) {
        float tt = 0, nn[3] = {0, 0, 0};
        int32_t ff = -1;
        int h = orc_query(m, o + 3 * i, d + 3 * i, max_t, &tt, &ff, nn);
        t[i] = h ? tt : nanf("");
        face[i] = h ? ff : -1;
        memcpy(nrm + 3 * i, nn, 12);
        hits += h;
    }
    return hits;
}
