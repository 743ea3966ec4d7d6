// terrain.h - ground contacts against a heightfield (hum_set_terrain): LowLevelHumanoidEnv(useCustomEnv=True)
// replaces HumanoidBulletEnv's plane with CustomScene's GEOM_HEIGHTFIELD body (/root/reference/humanoid.py:68-144).
//
// Geometry (Bullet btHeightfieldTerrainShape, upAxis z, PHY_FLOAT data, diamond subdivision, no flipped edges):
// vertex (i, j) at origin + scale * (i - (w-1)/2, j - (l-1)/2, h(i, j) - mid), mid = (min h + max h) / 2; cell
// (i, j) is split along (i,j)-(i+1,j+1) when i + j is even, along (i+1,j)-(i,j+1) otherwise.
// Contacts (the same sphere / capsule-end candidates as the plane): the closest point of the surface to the
// candidate's centre over the triangles of the (at most 2 x 2) cells within reach r + contact_thresh; a centre
// below the plane of the triangle under it takes that triangle's upward normal.  Restated the same way in
// oracle/physics_oracle.c (terrain_contact).  PyBullet parity unpinned, like the rest of the physics.
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

}  // namespace hk
