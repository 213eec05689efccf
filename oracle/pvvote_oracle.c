/*
 * pvvote_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the arithmetic of PVNet's RANSAC-voting CUDA kernels
 * (kennege/pvnet, lib/ransac_voting_gpu_layer/src/ransac_voting_kernel.cu,
 * cited below as KU:<line>).  It is the parity checker for the HIP library in
 * pvnet_amd/csrc and the CPU baseline leg of bench.py ("kind": "port").
 * Nothing in the product path links, loads or calls this file.
 *
 * Numerics contract:
 *   - IEEE-754 binary32, round-to-nearest, NO contraction (built with
 *     -ffp-contract=off, see Makefile), correctly rounded
 *     sqrtf and division, subnormals kept.
 *   - The `< 1e-6` guards compare a float against the double literal 1e-6,
 *     i.e. in double precision, exactly as the C++ source does (KU:42-43,121).
 *   - `angle_dist > inlier_thresh` is a float compare (KU:124).
 *
 * Pinning: the CUDA source cannot be built here (no nvcc; removed ATen APIs,
 * SURVEY.md 8(c)); this restatement is pinned by the tests/golden fixtures, which
 * tests/golden/make_golden.py produced by running the reference's own Python
 * voting layer with an independent torch-CPU restatement of the same kernels,
 * and by the LINEMOD-cat known answer (data/demo).
 */
/* contraction is disabled by -ffp-contract=off (Makefile) */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* KU:11-49 generate_hypothesis_kernel, one (h,v) pair. Returns 0 when the
 * pair is degenerate (the reference leaves the zero-initialised output). */
static int gen_one(const float *direct, const float *coords, const int32_t *idxs,
                   int vn, int hi, int vi, float *ox, float *oy)
{
    int t0 = idxs[hi * vn * 2 + vi * 2];
    int t1 = idxs[hi * vn * 2 + vi * 2 + 1];

    float nx0 = direct[t0 * vn * 2 + vi * 2 + 1];     /* KU:31-34 */
    float ny0 = -direct[t0 * vn * 2 + vi * 2];
    float cx0 = coords[t0 * 2];
    float cy0 = coords[t0 * 2 + 1];

    float nx1 = direct[t1 * vn * 2 + vi * 2 + 1];     /* KU:36-39 */
    float ny1 = -direct[t1 * vn * 2 + vi * 2];
    float cx1 = coords[t1 * 2];
    float cy1 = coords[t1 * 2 + 1];

    float d0 = nx1 * ny0 - nx0 * ny1;                 /* KU:42 */
    if ((double)fabsf(d0) < 1e-6) return 0;
    float d1 = ny1 * nx0 - ny0 * nx1;                 /* KU:43 */
    if ((double)fabsf(d1) < 1e-6) return 0;
    float p0 = nx0 * cx0 + ny0 * cy0;
    float p1 = nx1 * cx1 + ny1 * cy1;
    float y = (nx1 * p0 - nx0 * p1) / d0;             /* KU:44 */
    float x = (ny1 * p0 - ny0 * p1) / d1;             /* KU:45 */
    *ox = x;
    *oy = y;
    return 1;
}

void or_generate_hypothesis(const float *direct, const float *coords, const int32_t *idxs,
                            float *hypo, int tn, int vn, int hn)
{
    (void)tn;
    for (int hi = 0; hi < hn; ++hi)
        for (int vi = 0; vi < vn; ++vi) {
            float x = 0.f, y = 0.f;
            gen_one(direct, coords, idxs, vn, hi, vi, &x, &y);
            hypo[hi * vn * 2 + vi * 2] = x;           /* KU:47-48 (0 if skipped, KU:75) */
            hypo[hi * vn * 2 + vi * 2 + 1] = y;
        }
}

/* KU:107-125 voting_for_hypothesis_kernel, one (h,v,t) triple. */
static inline int vote_one(float nx, float ny, float cx, float cy, float hx, float hy, float thr)
{
    float dx = hx - cx;                               /* KU:116-117 */
    float dy = hy - cy;
    float norm1 = sqrtf(nx * nx + ny * ny);           /* KU:119 */
    float norm2 = sqrtf(dx * dx + dy * dy);           /* KU:120 */
    if ((double)norm1 < 1e-6 || (double)norm2 < 1e-6) return 0;  /* KU:121 */
    float angle_dist = (dx * nx + dy * ny) / (norm1 * norm2);    /* KU:123 */
    return angle_dist > thr;                          /* KU:124 */
}

int or_vote_test(float nx, float ny, float cx, float cy, float hx, float hy, float thr)
{
    return vote_one(nx, ny, cx, cy, hx, hy, thr);
}

/* Reference semantics: OR 1s into a caller-owned [hn,vn,tn] u8 tensor (KU:124-125). */
void or_voting_for_hypothesis(const float *direct, const float *coords, const float *hypo,
                              uint8_t *inliers, int tn, int vn, int hn, float thr)
{
    for (int hi = 0; hi < hn; ++hi)
        for (int vi = 0; vi < vn; ++vi) {
            float hx = hypo[hi * vn * 2 + vi * 2];
            float hy = hypo[hi * vn * 2 + vi * 2 + 1];
            uint8_t *row = inliers + ((int64_t)hi * vn + vi) * tn;
            for (int ti = 0; ti < tn; ++ti) {
                float cx = coords[ti * 2], cy = coords[ti * 2 + 1];
                float nx = direct[ti * vn * 2 + vi * 2], ny = direct[ti * vn * 2 + vi * 2 + 1];
                if (vote_one(nx, ny, cx, cy, hx, hy, thr)) row[ti] = 1;
            }
        }
}

/* counts[h][v] = sum_t inlier(h,v,t): what torch.sum(inlier, 2) returns
 * (ransac_voting_gpu.py:567) without materialising the mask. */
void or_vote_counts(const float *direct, const float *coords, const float *hypo,
                    int64_t *counts, int tn, int vn, int hn, float thr, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int hv = 0; hv < hn * vn; ++hv) {
        int hi = hv / vn, vi = hv % vn;
        float hx = hypo[hi * vn * 2 + vi * 2];
        float hy = hypo[hi * vn * 2 + vi * 2 + 1];
        int64_t c = 0;
        for (int ti = 0; ti < tn; ++ti) {
            float cx = coords[ti * 2], cy = coords[ti * 2 + 1];
            float nx = direct[ti * vn * 2 + vi * 2], ny = direct[ti * vn * 2 + vi * 2 + 1];
            c += vote_one(nx, ny, cx, cy, hx, hy, thr);
        }
        counts[hv] = c;
    }
    (void)nthreads;
}

/* KU:170-229 generate_hypothesis_vanishing_point_kernel. */
void or_generate_hypothesis_vp(const float *direct, const float *coords, const int32_t *idxs,
                               float *hypo, int tn, int vn, int hn)
{
    (void)tn;
    for (int hi = 0; hi < hn; ++hi)
        for (int vi = 0; vi < vn; ++vi) {
            int id0 = idxs[hi * vn * 2 + vi * 2];
            int id1 = idxs[hi * vn * 2 + vi * 2 + 1];
            float dx0 = direct[id0 * vn * 2 + vi * 2], dy0 = direct[id0 * vn * 2 + vi * 2 + 1];
            float cx0 = coords[id0 * 2], cy0 = coords[id0 * 2 + 1];
            float dx1 = direct[id1 * vn * 2 + vi * 2], dy1 = direct[id1 * vn * 2 + vi * 2 + 1];
            float cx1 = coords[id1 * 2], cy1 = coords[id1 * 2 + 1];
            float lx0 = dy0, ly0 = -dx0, lz0 = cy0 * dx0 - cx0 * dy0;   /* KU:201-203 */
            float lx1 = dy1, ly1 = -dx1, lz1 = cy1 * dx1 - cx1 * dy1;   /* KU:205-207 */
            float x = ly0 * lz1 - lz0 * ly1;                            /* KU:210-212 */
            float y = lz0 * lx1 - lx0 * lz1;
            float z = lx0 * ly1 - ly0 * lx1;
            float vx0 = dx0 * (x - z * cx0), vx1 = dx1 * (x - z * cx1); /* KU:215-218 */
            float vy0 = dy0 * (y - z * cy0), vy1 = dy1 * (y - z * cy1);
            if (vx0 < 0 && vx1 < 0 && vy0 < 0 && vy1 < 0) { z = -z; x = -x; y = -y; }  /* KU:220-221 */
            if (vx0 * vx1 < 0 || vy0 * vy1 < 0) { x = 0.f; y = 0.f; z = 0.f; }          /* KU:223-224 */
            hypo[hi * vn * 3 + vi * 3] = x;
            hypo[hi * vn * 3 + vi * 3 + 1] = y;
            hypo[hi * vn * 3 + vi * 3 + 2] = z;
        }
}

/* KU:268-310 voting_for_hypothesis_vanishing_point_kernel (OR-in semantics). */
void or_voting_for_hypothesis_vp(const float *direct, const float *coords, const float *hypo,
                                 uint8_t *inliers, int tn, int vn, int hn, float thr)
{
    for (int hi = 0; hi < hn; ++hi)
        for (int vi = 0; vi < vn; ++vi) {
            float hx = hypo[hi * vn * 3 + vi * 3];
            float hy = hypo[hi * vn * 3 + vi * 3 + 1];
            float hz = hypo[hi * vn * 3 + vi * 3 + 2];
            uint8_t *row = inliers + ((int64_t)hi * vn + vi) * tn;
            for (int ti = 0; ti < tn; ++ti) {
                float cx = coords[ti * 2], cy = coords[ti * 2 + 1];
                float ddx = direct[ti * vn * 2 + vi * 2], ddy = direct[ti * vn * 2 + vi * 2 + 1];
                float fx = hx - cx * hz;                                /* KU:297-298 */
                float fy = hy - cy * hz;
                float n1 = sqrtf(ddx * ddx + ddy * ddy);
                float n2 = sqrtf(fx * fx + fy * fy);
                if ((double)n1 < 1e-6 || (double)n2 < 1e-6) continue;   /* KU:302 */
                float ad = (ddx * fx + ddy * fy) / (n1 * n2);            /* KU:304 */
                float vx = fx * ddx, vy = fy * ddy;
                if (vx < 0 || vy < 0) continue;                          /* KU:307 */
                if (fabsf(ad) > thr) row[ti] = 1;                        /* KU:308-309 */
            }
        }
}

/* Mask threshold of generate_hypothesis' "skip" test, exposed so tests can
 * build degenerate pairs on purpose. */
int or_gen_one(const float *direct, const float *coords, const int32_t *idxs, int vn,
               int hi, int vi, float *ox, float *oy)
{
    return gen_one(direct, coords, idxs, vn, hi, vi, ox, oy);
}
