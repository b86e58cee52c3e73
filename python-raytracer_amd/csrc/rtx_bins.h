// rtx_bins.h — the pinhole projection of the primary-ray bins (rtx_api.hip primary_bins),
// shared by the host (spheres, boxes, hierarchy roots) and the device pass that bins a
// mesh's faces (rtx_bins.hip): the same fp64 operations in the same order on both, so the
// device bins are the host's bit for bit (tests/test_gpu_parity.py
// test_device_face_bins_equal_host).
//
// Every primary ray of a one-sample pinhole camera leaves one origin o toward
// x u + y v - d w (provided/scene.py:54, 60-61). A point p projects to the fractional
// column / row of the camera's own fp32 pixel tables xs / ys (scene.py:42, 48: the values
// the rays use, so no spacing estimate accumulates error across the image); a set of
// points, to the 8x8 bins its padded pixel rectangle covers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

namespace rtx {

#define RTX_BINS_HD __host__ __device__ __forceinline__

struct BinProj {
    double o[3];           // the rays' origin
    float u[3], v[3], w[3];  // the camera basis (ViewportCamera, fp32)
    double d;              // ViewportCamera.d
    const float* xs;       // [W] the strip's fp32 x table
    const float* ys;       // [H] the fp32 y table, bottom row first
    int32_t W, H;
};

struct BinRect {
    int32_t c0, c1, r0, r1;  // bin range (c0 > c1: off the strip)
};

// std::min / std::max as the host wrote them: (b < a) ? b : a
RTX_BINS_HD double bins_min(double a, double b) { return (b < a) ? b : a; }
RTX_BINS_HD double bins_max(double a, double b) { return (a < b) ? b : a; }

// fractional index of a screen coordinate x in the fp32 table t[n] (ascending)
RTX_BINS_HD double bins_table_pos(const float* t, int32_t n, double x) {
    if (x <= (double)t[0]) return (x - (double)t[0]) / ((double)t[1] - (double)t[0]);
    if (x >= (double)t[n - 1]) return (n - 1) + (x - (double)t[n - 1]) / ((double)t[n - 1] - (double)t[n - 2]);
    // std::upper_bound(t, t + n, (float)x): the first k with t[k-1] <= fl(x) < t[k]
    const float v = (float)x;
    int32_t lo = 0, hi = n;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (v < t[mid]) hi = mid;
        else lo = mid + 1;
    }
    const int32_t k1 = lo < 1 ? 1 : (lo > n - 1 ? n - 1 : lo);
    return (k1 - 1) + (x - (double)t[k1 - 1]) / ((double)t[k1] - (double)t[k1 - 1]);
}

// pixel coordinates (strip column, image row) and depth of p; false: grazing or behind
RTX_BINS_HD bool bins_project(const BinProj& P, const double p[3], double& col, double& row, double& depth) {
    double rel[3], len2 = 0.0, pu = 0.0, pv = 0.0, pw = 0.0;
    for (int a = 0; a < 3; ++a) {
        rel[a] = p[a] - P.o[a];
        len2 += rel[a] * rel[a];
        pu += rel[a] * P.u[a];
        pv += rel[a] * P.v[a];
        pw += rel[a] * P.w[a];
    }
    depth = -pw;
    if (!(depth > 1e-3 * sqrt(len2)) || !(depth > 1e-9)) return false;
    col = bins_table_pos(P.xs, P.W, P.d * pu / depth);
    row = (double)(P.H - 1) - bins_table_pos(P.ys, P.H, P.d * pv / depth);
    return true;
}

// bin range of the points' pixel rectangle padded by 2 pixels, and their least depth;
// false if a point cannot be projected
RTX_BINS_HD bool bins_rect(const BinProj& P, const double (*pts)[3], int n, BinRect& R, double& zlo) {
    double cmin = INFINITY, cmax = -INFINITY, rmin = INFINITY, rmax = -INFINITY;
    zlo = INFINITY;
    for (int i = 0; i < n; ++i) {
        double col, row, depth;
        if (!bins_project(P, pts[i], col, row, depth)) return false;
        cmin = bins_min(cmin, col); cmax = bins_max(cmax, col);
        rmin = bins_min(rmin, row); rmax = bins_max(rmax, row);
        zlo = bins_min(zlo, depth);
    }
    R = BinRect{1, 0, 1, 0};
    const double c0 = floor(cmin) - 2.0, c1 = ceil(cmax) + 2.0;
    const double r0 = floor(rmin) - 2.0, r1 = ceil(rmax) + 2.0;
    if (c1 >= 0.0 && c0 <= P.W - 1 && r1 >= 0.0 && r0 <= P.H - 1) {
        R.c0 = (int32_t)bins_max(0.0, c0) >> 3; R.c1 = (int32_t)bins_min((double)(P.W - 1), c1) >> 3;
        R.r0 = (int32_t)bins_max(0.0, r0) >> 3; R.r1 = (int32_t)bins_min((double)(P.H - 1), r1) >> 3;
    }
    return true;
}

// A face's depth bound as a bin entry stores it: fl32 rounded down (device and host)
RTX_BINS_HD float bins_zmin(double fz) {
    float z = (float)fz;
    if ((double)z > fz) z = nextafterf(z, -INFINITY);
    return z;
}

// The device face pass (rtx_bins.hip). Faces f of the mesh (triangle records of
// tri_stride floats, vertices v0 v1 v2 first) get their bin rectangles; the bins' face
// lists are laid out nearest first (stable by face index), as primary_bins does on the
// host. Buffers are the caller's (MeshBinsDev: sizes from mesh_bins_bytes).
struct MeshBinsDev {
    int4* rect;        // [n] per face
    double* fz;        // [n] depth bound per face
    int32_t* count;    // [nb] faces per bin, then [nb + 1] the fill cursor (start)
    int32_t* bad;      // [1] a face that cannot be projected
    uint64_t* keys;    // [n] fz bits, then sorted
    uint64_t* keys2;   // [n]
    int32_t* idx;      // [n] 0..n-1
    int32_t* order;    // [n] faces nearest first
    uint64_t* pairs;   // [npairs] (bin << 32 | rank)
    uint64_t* pairs2;  // [npairs]
    void* tmp;         // hipcub scratch
    size_t tmp_bytes;
};
// the sorts' one-time setup (rtx_scene_create of a scene with one mesh, so that the first
// camera upload does not pay it)
void mesh_bins_warm();
// device bytes of the first stage (faces n) and of the second (npairs), incl. scratch
size_t mesh_bins_bytes1(int32_t n, int32_t nb);
size_t mesh_bins_bytes2(int32_t n, int32_t npairs);
// stage 1: rectangles, depth bounds and per-bin counts (count[nb] zeroed first), the faces'
// nearest-first order; buf holds mesh_bins_bytes1. Fills m's stage-1 pointers.
hipError_t mesh_bins_stage1(const BinProj& P, const float* tris, int32_t tri_stride, int32_t n, int32_t bins_x,
                            int32_t nb, void* buf, MeshBinsDev& m, hipStream_t st);
// stage 2: with fill = the bins' start offsets (count[0..nb), overwritten), each face's
// bins get (bin, rank) pairs, sorted; faces_out[q] / zmin_out[q] for q < npairs. buf2
// holds mesh_bins_bytes2.
hipError_t mesh_bins_stage2(MeshBinsDev& m, int32_t n, int32_t bins_x, int32_t nb, int32_t npairs, void* buf2,
                            int32_t* faces_out, float* zmin_out, hipStream_t st);

}  // namespace rtx
