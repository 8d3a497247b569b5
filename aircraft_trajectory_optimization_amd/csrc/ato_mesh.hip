// ato_mesh.hip -- signed distance of points to a triangle mesh (the obstacle environment of
// scripts/obstacles.py). Replaces trimesh.proximity.signed_distance / closest_point as used by
// MeshObstacle (drone3d/obstacles/mesh_obstacle.py:38-41 signed_distance, :110-145 the tube's
// largest-empty-sphere search, :1312-1327 of base_raceline.py the collision check).
//
// One thread per query point, all triangles streamed through LDS in tiles (the mesh is small:
// 8884 triangles = 640 KB as fp64 edge form; every point needs every triangle, so the kernel
// is compute bound, ~80 flop per point-triangle pair):
//   * unsigned distance: closest point on each triangle (Voronoi-region test, Ericson,
//     Real-Time Collision Detection 5.1.5), minimum over the mesh
//   * sign: parity of the crossings of a fixed ray (Moller-Trumbore); odd = inside
// Result is positive outside, negative inside (MeshObstacle.signed_distance convention).
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
#include "../../include/ato.h"

struct ato_mesh {
    int nf = 0;
    double* d_tri = nullptr;   // [nf][9]: a, b - a, c - a
};

void ato_internal_set_error(const std::string& msg);   // ato_capi.hip: ato_last_error()

namespace {

int fail(int code, const std::string& m) {
    ato_internal_set_error(m);
    return code;
}

constexpr int TILE = 256;
// fixed, generic ray direction (not aligned with any mesh edge or face of an axis-aligned arena)
__constant__ double RAY[3] = {0.8017837257372732, 0.5345224838248488, 0.2672612419124244};

struct V3 {
    double x, y, z;
};
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 mul(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// closest point to p on triangle (a, a + ab, a + ac)
__device__ __forceinline__ V3 closest_on_triangle(V3 p, V3 a, V3 ab, V3 ac) {
    const V3 ap = sub(p, a);
    const double d1 = dot(ab, ap), d2 = dot(ac, ap);
    if (d1 <= 0.0 && d2 <= 0.0) return a;
    const V3 bp = sub(ap, ab);
    const double d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0.0 && d4 <= d3) return add(a, ab);
    const double vc = d1 * d4 - d3 * d2;
    if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) return add(a, mul(ab, d1 / (d1 - d3)));
    const V3 cp = sub(ap, ac);
    const double d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0.0 && d5 <= d6) return add(a, ac);
    const double vb = d5 * d2 - d1 * d6;
    if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) return add(a, mul(ac, d2 / (d2 - d6)));
    const double va = d3 * d6 - d5 * d4;
    if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
        const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        return add(add(a, ab), mul(sub(ac, ab), w));
    }
    const double den = 1.0 / (va + vb + vc);
    return add(a, add(mul(ab, vb * den), mul(ac, vc * den)));
}

// does the ray p + t RAY (t > 0) cross the triangle
__device__ __forceinline__ bool ray_hits(V3 p, V3 a, V3 ab, V3 ac) {
    const V3 d = {RAY[0], RAY[1], RAY[2]};
    const V3 pv = cross(d, ac);
    const double det = dot(ab, pv);
    if (fabs(det) < 1e-300) return false;
    const double inv = 1.0 / det;
    const V3 tv = sub(p, a);
    const double u = dot(tv, pv) * inv;
    if (u < 0.0 || u > 1.0) return false;
    const V3 qv = cross(tv, ab);
    const double v = dot(d, qv) * inv;
    if (v < 0.0 || u + v > 1.0) return false;
    return dot(ac, qv) * inv > 0.0;
}

__global__ __launch_bounds__(TILE) void k_mesh_sdist(int n, const double* __restrict__ pts, int nf,
                                                    const double* __restrict__ tri, double* __restrict__ dist,
                                                    double* __restrict__ closest) {
    __shared__ double tile[TILE * 9];
    const int i = blockIdx.x * TILE + threadIdx.x;
    const bool live = i < n;
    const V3 p = live ? V3{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]} : V3{0, 0, 0};
    double best = 1e300;
    V3 bq = p;
    int crossings = 0;
    for (int t0 = 0; t0 < nf; t0 += TILE) {
        const int cnt = min(TILE, nf - t0);
        __syncthreads();
        for (int e = threadIdx.x; e < cnt * 9; e += TILE) tile[e] = tri[(long)t0 * 9 + e];
        __syncthreads();
        if (live) {
            for (int t = 0; t < cnt; ++t) {
                const double* q = tile + t * 9;
                const V3 a = {q[0], q[1], q[2]}, ab = {q[3], q[4], q[5]}, ac = {q[6], q[7], q[8]};
                const V3 c = closest_on_triangle(p, a, ab, ac);
                const V3 dv = sub(p, c);
                const double d2 = dot(dv, dv);
                if (d2 < best) {
                    best = d2;
                    bq = c;
                }
                crossings += ray_hits(p, a, ab, ac) ? 1 : 0;
            }
        }
    }
    if (!live) return;
    const double d = sqrt(best);
    dist[i] = (crossings & 1) ? -d : d;
    if (closest) {
        closest[3 * i] = bq.x;
        closest[3 * i + 1] = bq.y;
        closest[3 * i + 2] = bq.z;
    }
}

}  // namespace

extern "C" {

int ato_mesh_create(const double* vertices, int32_t n_vertices, const int32_t* faces, int32_t n_faces,
                    ato_mesh** out) {
    if (!vertices || !faces || !out || n_vertices < 3 || n_faces < 1) return fail(ATO_ERR_ARG, "bad mesh arguments");
    std::vector<double> tri((size_t)n_faces * 9);
    for (int f = 0; f < n_faces; ++f) {
        int idx[3];
        for (int j = 0; j < 3; ++j) {
            idx[j] = faces[3 * f + j];
            if (idx[j] < 0 || idx[j] >= n_vertices) return fail(ATO_ERR_ARG, "face index out of range");
        }
        for (int c = 0; c < 3; ++c) {
            const double a = vertices[3 * idx[0] + c];
            tri[(size_t)f * 9 + c] = a;
            tri[(size_t)f * 9 + 3 + c] = vertices[3 * idx[1] + c] - a;
            tri[(size_t)f * 9 + 6 + c] = vertices[3 * idx[2] + c] - a;
        }
    }
    auto* m = new ato_mesh();
    m->nf = n_faces;
    if (hipMalloc(&m->d_tri, tri.size() * sizeof(double)) != hipSuccess ||
        hipMemcpy(m->d_tri, tri.data(), tri.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(m->d_tri);
        delete m;
        return fail(ATO_ERR_HIP, "mesh upload failed");
    }
    *out = m;
    return ATO_OK;
}

int ato_mesh_destroy(ato_mesh* m) {
    if (!m) return ATO_OK;
    (void)hipFree(m->d_tri);
    delete m;
    return ATO_OK;
}

int ato_mesh_signed_distance(ato_mesh* m, int32_t n, const double* points, double* dist, double* closest,
                             void* stream) {
    if (!m || n < 0 || (n > 0 && (!points || !dist))) return fail(ATO_ERR_ARG, "bad distance arguments");
    if (n == 0) return ATO_OK;
    hipLaunchKernelGGL(k_mesh_sdist, dim3((n + TILE - 1) / TILE), dim3(TILE), 0, (hipStream_t)stream, n, points,
                       m->nf, (const double*)m->d_tri, dist, closest);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ATO_OK : fail(ATO_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
