// The primary-ray face bins of a mesh, built on the device (rtx_api.hip rtx_camera_set):
// per face its pinhole rectangle of 8x8 bins and depth bound (rtx_bins.h, the host's
// arithmetic), the faces in nearest-first order (a stable radix sort of the depth bounds),
// and every bin's face list in that order (a radix sort of (bin, rank) pairs). The host
// version walked 81,920 faces, three table searches each, and sorted them on one core
// (~20 ms per camera of the 81,920-face mesh); here it is a few short kernels.
// A translation unit of its own: rocPRIM's sorts compile slowly and in parallel.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include "rtx_bins.h"

namespace rtx {
namespace {

size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

// One thread per face: its bin rectangle, depth bound and bin counts.
__global__ __launch_bounds__(256) void k_face_rects(BinProj P, const float* __restrict__ tris, int32_t stride, int32_t n,
                                                    int32_t bins_x, int4* __restrict__ rect, double* __restrict__ fz,
                                                    uint64_t* __restrict__ keys, int32_t* __restrict__ idx,
                                                    int32_t* __restrict__ count, int32_t* __restrict__ bad) {
    const int32_t f = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (f >= n) return;
    const float* T = tris + (int64_t)f * stride;
    double pts[3][3];
    for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 3; ++a) pts[k][a] = T[3 * k + a];
    BinRect R;
    double zlo;
    idx[f] = f;
    if (!bins_rect(P, pts, 3, R, zlo)) {
        atomicOr(bad, 1);
        rect[f] = make_int4(1, 0, 1, 0);
        fz[f] = 0.0;
        keys[f] = 0ull;
        return;
    }
    rect[f] = make_int4(R.c0, R.c1, R.r0, R.r1);
    const double z = zlo * (1.0 - 1e-4);  // (primary_bins: below every t on the face)
    fz[f] = z;
    keys[f] = __double_as_longlong(z) ^ (z < 0.0 ? ~0ull : 0ull) ^ (z < 0.0 ? 0ull : 0x8000000000000000ull);
    for (int32_t by = R.r0; by <= R.r1; ++by)
        for (int32_t bx = R.c0; bx <= R.c1; ++bx) atomicAdd(&count[by * bins_x + bx], 1);
}

// One thread per rank r (the r-th nearest face): a (bin, r) pair in each of its bins.
__global__ __launch_bounds__(256) void k_face_pairs(const int32_t* __restrict__ order, const int4* __restrict__ rect,
                                                    int32_t n, int32_t bins_x, int32_t* __restrict__ fill,
                                                    uint64_t* __restrict__ pairs) {
    const int32_t r = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (r >= n) return;
    const int4 R = rect[order[r]];
    for (int32_t by = R.z; by <= R.w; ++by)
        for (int32_t bx = R.x; bx <= R.y; ++bx) {
            const int32_t b = by * bins_x + bx;
            const int32_t q = atomicAdd(&fill[b], 1);
            pairs[q] = ((uint64_t)(uint32_t)b << 32) | (uint32_t)r;
        }
}

// One thread per list entry q: the face and its depth bound.
__global__ __launch_bounds__(256) void k_face_lists(const uint64_t* __restrict__ pairs, const int32_t* __restrict__ order,
                                                    const double* __restrict__ fz, int32_t np,
                                                    int32_t* __restrict__ faces, float* __restrict__ zmin) {
    const int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= np) return;
    const int32_t f = order[(uint32_t)pairs[q]];
    faces[q] = f;
    zmin[q] = bins_zmin(fz[f]);
}

int bit_width(uint32_t x) {
    int b = 0;
    while (x) { ++b; x >>= 1; }
    return b;
}

size_t sort_pairs_tmp(int32_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, n);
    return bytes;
}
size_t sort_keys_tmp(int32_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, n);
    return bytes;
}

}  // namespace

void mesh_bins_warm() {
    // The first sort of a process costs ~8 ms (profiles/r06/s3/setup_blob.err: rocPRIM
    // reads the device's properties with hipGetDeviceProperties and clears its scan state
    // with hipMemsetAsync, whose blit kernels the runtime loads on first use): one tiny
    // sort of each kind, here, so that the first camera upload does not pay it.
    constexpr int32_t n = 256;
    const size_t tp = sort_pairs_tmp(n), tk = sort_keys_tmp(n);
    const size_t bytes = 4 * align256(sizeof(uint64_t) * n) + align256(tp) + align256(tk);
    char* p = nullptr;
    if (hipMalloc((void**)&p, bytes) != hipSuccess) return;
    uint64_t* k0 = reinterpret_cast<uint64_t*>(p);
    uint64_t* k1 = reinterpret_cast<uint64_t*>(p + align256(sizeof(uint64_t) * n));
    int32_t* v0 = reinterpret_cast<int32_t*>(p + 2 * align256(sizeof(uint64_t) * n));
    int32_t* v1 = reinterpret_cast<int32_t*>(p + 3 * align256(sizeof(uint64_t) * n));
    char* t = p + 4 * align256(sizeof(uint64_t) * n);
    size_t tpb = tp, tkb = tk;
    if (hipMemsetAsync(p, 0, 4 * align256(sizeof(uint64_t) * n), nullptr) == hipSuccess &&
        hipcub::DeviceRadixSort::SortPairs(t, tpb, k0, k1, v0, v1, n, 0, 64, nullptr) == hipSuccess)
        (void)hipcub::DeviceRadixSort::SortKeys(t + align256(tp), tkb, k0, k1, n, 0, 64, nullptr);
    (void)hipStreamSynchronize(nullptr);
    (void)hipFree(p);
}

size_t mesh_bins_bytes1(int32_t n, int32_t nb) {
    return align256(sizeof(int4) * n) + align256(sizeof(double) * n) + align256(sizeof(int32_t) * (nb + 1)) +
           align256(sizeof(int32_t)) + 2 * align256(sizeof(uint64_t) * n) + 2 * align256(sizeof(int32_t) * n) +
           align256(sort_pairs_tmp(n));
}

size_t mesh_bins_bytes2(int32_t n, int32_t npairs) {
    (void)n;
    return 2 * align256(sizeof(uint64_t) * (size_t)npairs) + align256(sort_keys_tmp(npairs));
}

hipError_t mesh_bins_stage1(const BinProj& P, const float* tris, int32_t tri_stride, int32_t n, int32_t bins_x,
                            int32_t nb, void* buf, MeshBinsDev& m, hipStream_t st) {
    char* p = static_cast<char*>(buf);
    auto take = [&](size_t bytes) {
        void* q = p;
        p += align256(bytes);
        return q;
    };
    m.rect = static_cast<int4*>(take(sizeof(int4) * n));
    m.fz = static_cast<double*>(take(sizeof(double) * n));
    m.count = static_cast<int32_t*>(take(sizeof(int32_t) * (nb + 1)));
    m.bad = static_cast<int32_t*>(take(sizeof(int32_t)));
    m.keys = static_cast<uint64_t*>(take(sizeof(uint64_t) * n));
    m.keys2 = static_cast<uint64_t*>(take(sizeof(uint64_t) * n));
    m.idx = static_cast<int32_t*>(take(sizeof(int32_t) * n));
    m.order = static_cast<int32_t*>(take(sizeof(int32_t) * n));
    m.tmp_bytes = sort_pairs_tmp(n);
    m.tmp = take(m.tmp_bytes);
    hipError_t e = hipMemsetAsync(m.count, 0, sizeof(int32_t) * (nb + 1), st);
    if (e == hipSuccess) e = hipMemsetAsync(m.bad, 0, sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    if (n > 0) {
        hipLaunchKernelGGL(k_face_rects, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P, tris, tri_stride, n,
                           bins_x, m.rect, m.fz, m.keys, m.idx, m.count, m.bad);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // nearest first; a stable sort keeps equal bounds in face order (std::stable_sort)
        e = hipcub::DeviceRadixSort::SortPairs(m.tmp, m.tmp_bytes, m.keys, m.keys2, m.idx, m.order, n, 0, 64, st);
    }
    return e;
}

hipError_t mesh_bins_stage2(MeshBinsDev& m, int32_t n, int32_t bins_x, int32_t nb, int32_t npairs, void* buf2,
                            int32_t* faces_out, float* zmin_out, hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    char* p = static_cast<char*>(buf2);
    m.pairs = reinterpret_cast<uint64_t*>(p);
    p += align256(sizeof(uint64_t) * (size_t)npairs);
    m.pairs2 = reinterpret_cast<uint64_t*>(p);
    p += align256(sizeof(uint64_t) * (size_t)npairs);
    size_t tmp_bytes = sort_keys_tmp(npairs);
    hipLaunchKernelGGL(k_face_pairs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, m.order, m.rect, n, bins_x,
                       m.count, m.pairs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // (bin, rank) order: each bin's list nearest first (the bins' lengths are the counts,
    // so its entries land at [start, start + count)); the bits above the bin index are 0
    e = hipcub::DeviceRadixSort::SortKeys(p, tmp_bytes, m.pairs, m.pairs2, npairs, 0, 32 + bit_width((uint32_t)nb), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_face_lists, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, m.pairs2, m.order, m.fz,
                       npairs, faces_out, zmin_out);
    return hipGetLastError();
}

}  // namespace rtx
