// terrain.h - ground contacts against a heightfield (hum_set_terrain): LowLevelHumanoidEnv(useCustomEnv=True)
// replaces HumanoidBulletEnv's plane with CustomScene's GEOM_HEIGHTFIELD body (/root/reference/humanoid.py:68-144).
//
// Geometry (Bullet btHeightfieldTerrainShape, upAxis z, PHY_FLOAT data, diamond subdivision, no flipped edges):
// vertex (i, j) at origin + scale * (i - (w-1)/2, j - (l-1)/2, h(i, j) - mid), mid = (min h + max h) / 2; cell
// (i, j) is split along (i,j)-(i+1,j+1) when i + j is even, along (i+1,j)-(i,j+1) otherwise.
// Contacts (the same sphere / capsule-end candidates as the plane): the closest point of the surface to the
// candidate's centre over the triangles of the (at most 2 x 2) cells within reach r + contact_thresh; a centre
// below the plane of the triangle under it takes that triangle's upward normal.  Capsule bodies additionally touch
// the terrain's convex edges (ridge_contacts below: the local minima of the axis-to-surface distance inside the
// axis).  Restated the same way in oracle/physics_oracle.c (terrain_contact, ridge_contacts).  PyBullet parity
// unpinned, like the rest of the physics.
#pragma once
#include "physics.h"

namespace hk {

__host__ __device__ inline unsigned long long tsplitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// the terrain of a lane's next episode: chained from its previous terrain key and its RNG stream key, so every
// reset (CustomScene.episode_restart) yields a new terrain whatever the reset draws
constexpr unsigned long long TERRAIN_SALT = 0x2545F4914F6CDD1Dull;
__host__ __device__ inline unsigned long long next_terrain_key(unsigned long long prev, unsigned long long rng_key) {
    return tsplitmix64(prev ^ rng_key ^ TERRAIN_SALT);
}
// CustomScene.episode_restart (humanoid.py:94-111): each 2 x 2 vertex block at random.uniform(0, 0.05) * 10, the
// four centre blocks (63..64 x 63..64) at 0; the uniform is a 53-bit counter-based draw (key + block index)
__host__ __device__ inline float random_block_height(unsigned long long key, int bi, int bj) {
    if ((bi == 63 || bi == 64) && (bj == 63 || bj == 64)) return 0.f;
    const unsigned long long x = tsplitmix64(key + (unsigned long long)(bi + 128 * bj));
    const double u = (double)(x >> 11) * 0x1.0p-53;
    return (float)((0.05 * u) * 10.0);
}

template <typename T>
__device__ inline void terrain_vertex(const PhysParams& P, unsigned long long key, int i, int j, T* v) {
    const float h = P.terrain == 1 ? P.hf[i + j * P.hf_w] : random_block_height(key, i >> 1, j >> 1);
    v[0] = ((T)i - (T)(0.5 * (P.hf_w - 1))) * (T)P.hf_s[0] + (T)P.hf_o[0];
    v[1] = ((T)j - (T)(0.5 * (P.hf_l - 1))) * (T)P.hf_s[1] + (T)P.hf_o[1];
    v[2] = ((T)h - (T)P.hf_mid) * (T)P.hf_s[2] + (T)P.hf_o[2];
}

// closest point of triangle (a, b, c) to p (Ericson, Real-Time Collision Detection 5.1.5)
template <typename T>
__device__ inline void closest_on_triangle(const T* p, const T* a, const T* b, const T* c, T* q) {
    T ab[3], ac[3], ap[3];
#pragma unroll
    for (int k = 0; k < 3; k++) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ap[k] = p[k] - a[k]; }
    const T d1 = dot3(ab, ap), d2 = dot3(ac, ap);
    if (d1 <= T(0) && d2 <= T(0)) { for (int k = 0; k < 3; k++) q[k] = a[k]; return; }
    T bp[3];
#pragma unroll
    for (int k = 0; k < 3; k++) bp[k] = p[k] - b[k];
    const T d3 = dot3(ab, bp), d4 = dot3(ac, bp);
    if (d3 >= T(0) && d4 <= d3) { for (int k = 0; k < 3; k++) q[k] = b[k]; return; }
    const T vc = d1 * d4 - d3 * d2;
    if (vc <= T(0) && d1 >= T(0) && d3 <= T(0)) {
        const T t = d1 / (d1 - d3);
        for (int k = 0; k < 3; k++) q[k] = a[k] + t * ab[k];
        return;
    }
    T cp[3];
#pragma unroll
    for (int k = 0; k < 3; k++) cp[k] = p[k] - c[k];
    const T d5 = dot3(ab, cp), d6 = dot3(ac, cp);
    if (d6 >= T(0) && d5 <= d6) { for (int k = 0; k < 3; k++) q[k] = c[k]; return; }
    const T vb = d5 * d2 - d1 * d6;
    if (vb <= T(0) && d2 >= T(0) && d6 <= T(0)) {
        const T t = d2 / (d2 - d6);
        for (int k = 0; k < 3; k++) q[k] = a[k] + t * ac[k];
        return;
    }
    const T va = d3 * d6 - d5 * d4;
    if (va <= T(0) && (d4 - d3) >= T(0) && (d5 - d6) >= T(0)) {
        const T t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        for (int k = 0; k < 3; k++) q[k] = b[k] + t * (c[k] - b[k]);
        return;
    }
    const T den = T(1) / (va + vb + vc);
    const T v = vb * den, w = vc * den;
    for (int k = 0; k < 3; k++) q[k] = a[k] + ab[k] * v + ac[k] * w;
}

// the two triangles of cell (ci, cj) (t = 0, 1), vertex index offsets (di, dj) per corner
__host__ __device__ inline void cell_triangle(int ci, int cj, int t, int* di, int* dj) {
    const bool diag00 = !((ci + cj) & 1);   // split along (i,j)-(i+1,j+1)
    // diag00: (0,0),(0,1),(1,1) | (0,0),(1,1),(1,0); else: (0,0),(0,1),(1,0) | (1,0),(0,1),(1,1)
    const int A[2][2][6] = {{{0, 0, 1, 0, 1, 1}, {0, 1, 1, 0, 1, 0}}, {{0, 0, 1, 0, 1, 0}, {1, 0, 1, 0, 1, 1}}};
    const int* o = A[diag00 ? 0 : 1][t];   // di = o[0..2], dj = o[3..5]
    for (int k = 0; k < 3; k++) { di[k] = o[k]; dj[k] = o[3 + k]; }
}

// sphere (centre c, radius r) vs the terrain: true with the contact normal n (terrain -> sphere) and signed
// distance d when d < contact_thresh
template <typename T>
__device__ inline bool terrain_contact(const PhysParams& P, unsigned long long key, const T* c, T r, T* n, T& d) {
    const T sx = (T)P.hf_s[0], sy = (T)P.hf_s[1];
    T u = (c[0] - (T)P.hf_o[0]) / sx + (T)(0.5 * (P.hf_w - 1));
    T v = (c[1] - (T)P.hf_o[1]) / sy + (T)(0.5 * (P.hf_l - 1));
    if (!(u > T(-2) && u < (T)(P.hf_w + 1) && v > T(-2) && v < (T)(P.hf_l + 1))) return false;   // off the grid / NaN
    const T reach = r + (T)P.contact_thresh;
    int i0 = (int)floor(u - reach / sx), i1 = (int)floor(u + reach / sx);
    int j0 = (int)floor(v - reach / sy), j1 = (int)floor(v + reach / sy);
    i0 = i0 < 0 ? 0 : i0;
    j0 = j0 < 0 ? 0 : j0;
    i1 = i1 > P.hf_w - 2 ? P.hf_w - 2 : i1;
    j1 = j1 > P.hf_l - 2 ? P.hf_l - 2 : j1;
    if (i0 > i1 || j0 > j1) return false;
    T best = T(-1), q[3] = {0, 0, 0};
#pragma unroll 1
    for (int cj = j0; cj <= j1; cj++)
#pragma unroll 1
        for (int ci = i0; ci <= i1; ci++)
#pragma unroll 1
            for (int t = 0; t < 2; t++) {
                int di[3], dj[3];
                cell_triangle(ci, cj, t, di, dj);
                T va[3], vb[3], vc[3], qq[3], dv[3];
                terrain_vertex(P, key, ci + di[0], cj + dj[0], va);
                terrain_vertex(P, key, ci + di[1], cj + dj[1], vb);
                terrain_vertex(P, key, ci + di[2], cj + dj[2], vc);
                closest_on_triangle(c, va, vb, vc, qq);
                for (int k = 0; k < 3; k++) dv[k] = c[k] - qq[k];
                const T d2 = dot3(dv, dv);
                if (best < T(0) || d2 < best) {
                    best = d2;
                    for (int k = 0; k < 3; k++) q[k] = qq[k];
                }
            }
    // the triangle under the centre: below its plane = inside the terrain
    T nf[3] = {0, 0, 1}, sd = T(1);
    const int fi = (int)floor(u), fj = (int)floor(v);
    if (fi >= 0 && fi <= P.hf_w - 2 && fj >= 0 && fj <= P.hf_l - 2) {
        const T fa = u - (T)fi, fb = v - (T)fj;
        const int t = !((fi + fj) & 1) ? (fb >= fa ? 0 : 1) : (fa + fb <= T(1) ? 0 : 1);
        int di[3], dj[3];
        cell_triangle(fi, fj, t, di, dj);
        T va[3], vb[3], vc[3], e1[3], e2[3], ap[3];
        terrain_vertex(P, key, fi + di[0], fj + dj[0], va);
        terrain_vertex(P, key, fi + di[1], fj + dj[1], vb);
        terrain_vertex(P, key, fi + di[2], fj + dj[2], vc);
        for (int k = 0; k < 3; k++) { e1[k] = vb[k] - va[k]; e2[k] = vc[k] - va[k]; ap[k] = c[k] - va[k]; }
        cross3(e1, e2, nf);
        const T il = (nf[2] < T(0) ? T(-1) : T(1)) / sqrt(dot3(nf, nf));
        for (int k = 0; k < 3; k++) nf[k] *= il;
        sd = dot3(ap, nf);
    }
    if (sd < T(0)) {
        for (int k = 0; k < 3; k++) n[k] = nf[k];
        d = sd - r;
    } else {
        const T dist = sqrt(best);
        if (dist <= (T)1e-9) {
            for (int k = 0; k < 3; k++) n[k] = nf[k];
            d = -r;
        } else {
            const T id = T(1) / dist;
            for (int k = 0; k < 3; k++) n[k] = (c[k] - q[k]) * id;
            d = dist - r;
        }
    }
    return d < (T)P.contact_thresh;
}

// closest points of segments p1q1 / p2q2 with their parameters (physics.h seg_seg's clamping, exact divisions)
template <typename T>
__device__ inline void seg_seg_st(const T* p1, const T* q1, const T* p2, const T* q2, T* c1, T* c2, T& s, T& t) {
    T d1[3], d2[3], r[3];
#pragma unroll
    for (int i = 0; i < 3; i++) { d1[i] = q1[i] - p1[i]; d2[i] = q2[i] - p2[i]; r[i] = p1[i] - p2[i]; }
    const T a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    const T EPS = (T)1e-12;
    if (a <= EPS && e <= EPS) { s = t = 0; }
    else if (a <= EPS) { s = 0; t = clampT(f / e, T(0), T(1)); }
    else {
        const T c = dot3(d1, r);
        if (e <= EPS) { t = 0; s = clampT(-c / a, T(0), T(1)); }
        else {
            const T b = dot3(d1, d2), den = a * e - b * b;
            s = (den > EPS) ? clampT((b * f - c * e) / den, T(0), T(1)) : T(0);
            t = (b * s + f) / e;
            if (t < 0) { t = 0; s = clampT(-c / a, T(0), T(1)); }
            else if (t > 1) { t = 1; s = clampT((b - c) / a, T(0), T(1)); }
        }
    }
#pragma unroll
    for (int i = 0; i < 3; i++) { c1[i] = p1[i] + d1[i] * s; c2[i] = p2[i] + d2[i] * t; }
}

// Capsule bodies against the heightfield (oracle/physics_oracle.c ridge_contacts, where the model is argued):
// Bullet's convex-concave collision gives a capsule a closest-point contact per triangle under it, kept in one
// 4-point manifold; restated statelessly as the local minima of the axis-to-surface distance.  Over a facet that
// distance is linear along the axis and across a concave edge it is the minimum of two linear functions, so the
// minima are the axis ends (the end-cap candidates above) and the points where the axis passes over a CONVEX edge.
// For each interior grid edge within reach whose two triangles meet convexly (the far vertex of the second more
// than RIDGE_FLAT below the first's plane): (s, e) = closest points of axis and edge; kept when s is more than the
// breaking threshold from both axis ends, when no facet is closer to s than |s - e| - RIDGE_TOL (or s lies inside
// the terrain), and when terrain_contact at s is in range - the contact is terrain_contact's at s.  A candidate within
// the breaking threshold of a kept one is dropped; at most RIDGE_MAX per capsule (with the two end caps, Bullet's
// 4-point manifold), a deeper one replacing the shallowest kept.  Edge walk: vertex rows j, vertices i, then the
// horizontal, vertical and diagonal edge anchored at vertex (i, j).  Returns the count; per kept contact the normal,
// signed distance and axis parameter t.
constexpr int RIDGE_MAX = 2;
template <typename T>
__device__ inline int ridge_contacts(const PhysParams& P, unsigned long long key, const T* a, const T* b, T r,
                                     T (*rn)[3], T* rd, T* rt) {
    const T RIDGE_BREAK = (T)0.02, RIDGE_TOL = (T)1e-5, RIDGE_FLAT = (T)1e-5;
    const T sx = (T)P.hf_s[0], sy = (T)P.hf_s[1], cw = (T)(0.5 * (P.hf_w - 1)), cl = (T)(0.5 * (P.hf_l - 1));
    const T ua = (a[0] - (T)P.hf_o[0]) / sx + cw, ub = (b[0] - (T)P.hf_o[0]) / sx + cw;
    const T va = (a[1] - (T)P.hf_o[1]) / sy + cl, vb = (b[1] - (T)P.hf_o[1]) / sy + cl;
    if (!(ua > T(-2) && ua < (T)(P.hf_w + 1) && va > T(-2) && va < (T)(P.hf_l + 1) && ub > T(-2) &&
          ub < (T)(P.hf_w + 1) && vb > T(-2) && vb < (T)(P.hf_l + 1))) return 0;
    T ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    const T len = sqrt(dot3(ab, ab));
    if (len <= T(2) * RIDGE_BREAK) return 0;
    const T reach = r + (T)P.contact_thresh;
    int i0 = (int)floor((ua < ub ? ua : ub) - reach / sx), i1 = (int)floor((ua > ub ? ua : ub) + reach / sx);
    int j0 = (int)floor((va < vb ? va : vb) - reach / sy), j1 = (int)floor((va > vb ? va : vb) + reach / sy);
    i0 = i0 < 0 ? 0 : i0;
    j0 = j0 < 0 ? 0 : j0;
    i1 = i1 > P.hf_w - 2 ? P.hf_w - 2 : i1;
    j1 = j1 > P.hf_l - 2 ? P.hf_l - 2 : j1;
    int nk = 0;
#pragma unroll 1
    for (int j = j0; j <= j1 + 1; j++)
#pragma unroll 1
        for (int i = i0; i <= i1 + 1; i++)
#pragma unroll 1
            for (int kind = 0; kind < 3; kind++) {
                const bool even = !((i + j) & 1);
                int ev[4][2];   // edge (0, 1) and the far vertices of its two triangles (diamond subdivision)
                if (kind == 0) {   // horizontal (i, j)-(i+1, j): cells (i, j-1) and (i, j)
                    if (i > i1 || j < 1 || j > P.hf_l - 2) continue;
                    ev[0][0] = i; ev[0][1] = j; ev[1][0] = i + 1; ev[1][1] = j;
                    ev[2][0] = even ? i + 1 : i; ev[2][1] = j + 1; ev[3][0] = even ? i + 1 : i; ev[3][1] = j - 1;
                } else if (kind == 1) {   // vertical (i, j)-(i, j+1): cells (i-1, j) and (i, j)
                    if (j > j1 || i < 1 || i > P.hf_w - 2) continue;
                    ev[0][0] = i; ev[0][1] = j; ev[1][0] = i; ev[1][1] = j + 1;
                    ev[2][0] = i + 1; ev[2][1] = even ? j + 1 : j; ev[3][0] = i - 1; ev[3][1] = even ? j + 1 : j;
                } else {   // the diagonal of cell (i, j)
                    if (i > i1 || j > j1) continue;
                    ev[0][0] = even ? i : i + 1; ev[0][1] = j; ev[1][0] = even ? i + 1 : i; ev[1][1] = j + 1;
                    ev[2][0] = i; ev[2][1] = even ? j + 1 : j; ev[3][0] = i + 1; ev[3][1] = even ? j : j + 1;
                }
                T A[3], B[3], C1[3], C2[3], e1[3], f1[3], g2[3], n1[3];
                terrain_vertex(P, key, ev[0][0], ev[0][1], A);
                terrain_vertex(P, key, ev[1][0], ev[1][1], B);
                terrain_vertex(P, key, ev[2][0], ev[2][1], C1);
                terrain_vertex(P, key, ev[3][0], ev[3][1], C2);
#pragma unroll
                for (int k = 0; k < 3; k++) { e1[k] = B[k] - A[k]; f1[k] = C1[k] - A[k]; g2[k] = C2[k] - A[k]; }
                cross3(e1, f1, n1);
                T conv = dot3(g2, n1);
                if (n1[2] < T(0)) conv = -conv;
                if (!(conv < -RIDGE_FLAT * sqrt(dot3(n1, n1)))) continue;   // flat or concave
                T sp[3], ep[3], t, u;
                seg_seg_st(a, b, A, B, sp, ep, t, u);
                if (!(t * len > RIDGE_BREAK && (T(1) - t) * len > RIDGE_BREAK)) continue;
                const T dv[3] = {sp[0] - ep[0], sp[1] - ep[1], sp[2] - ep[2]};
                const T dse = sqrt(dot3(dv, dv));
                if (!(dse - r < (T)P.contact_thresh)) continue;
                T n[3], d;
                if (!terrain_contact<T>(P, key, sp, r, n, d)) continue;
                if (!(d + r < T(0) || d + r >= dse - RIDGE_TOL)) continue;   // a facet is closer: not a minimum
                bool dup = false;
                for (int k = 0; k < nk; k++)
                    if (fabs(rt[k] - t) * len < RIDGE_BREAK) dup = true;
                if (dup) continue;
                int slot = nk;
                if (nk == RIDGE_MAX) {
                    slot = rd[0] >= rd[1] ? 0 : 1;
                    if (!(d < rd[slot])) continue;
                } else {
                    nk++;
                }
#pragma unroll
                for (int k = 0; k < 3; k++) rn[slot][k] = n[k];
                rd[slot] = d;
                rt[slot] = t;
            }
    return nk;
}

}  // namespace hk
