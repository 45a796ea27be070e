// Probe: HBM rate of the full-cov update's p/m/v traffic (read + write 3
// arrays, 4.72 M floats each) in (a) the update kernel's tile pattern
// (64-row band x 64-column block, each row a 256-byte run of the packed
// triangle, float4 per lane, 4 rows per wave instruction), (b) whole-band
// row-contiguous sweeps (64-row band, each WG walks its rows' full length),
// (c) plain contiguous streaming of the same bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
struct Tile { int r0, c0; };
__global__ __launch_bounds__(256) void tiles(const Tile* t, float* p, float* m, float* v, int n) {
    const Tile tt = t[blockIdx.x];
    const int col4 = threadIdx.x & 15, srow = threadIdx.x >> 4;
    for (int j = 0; j < 4; ++j) {
        const int r = tt.r0 + srow + 16 * j;
        const int c = tt.c0 + 4 * col4;
        if (r >= n - 1 || c >= r) continue;
        const long o = (long)r * (r - 1) / 2 + c;
        if (c + 3 < r) {
            float4 a = *(float4*)(p + o), b = *(float4*)(m + o), d = *(float4*)(v + o);
            a.x += 1; b.y += 1; d.z += 1;
            *(float4*)(p + o) = a; *(float4*)(m + o) = b; *(float4*)(v + o) = d;
        } else {
            for (int i = 0; c + i < r; ++i) { p[o + i] += 1; m[o + i] += 1; v[o + i] += 1; }
        }
    }
}
// aligned windows: row r of tile k covers columns [64k - d_r, 64k + 64 - d_r),
// d_r = (r(r-1)/2) mod 32, so every row run starts on a 128-byte line
__global__ __launch_bounds__(256) void atiles(const Tile* t, float* p, float* m, float* v, int n) {
    const Tile tt = t[blockIdx.x];
    const int col4 = threadIdx.x & 15, srow = threadIdx.x >> 4;
    for (int j = 0; j < 4; ++j) {
        const int r = tt.r0 + srow + 16 * j;
        if (r >= n - 1) continue;
        const long base = (long)r * (r - 1) / 2;
        const int d = (int)(base & 31);
        const int c = tt.c0 - d + 4 * col4;
        if (c >= r || c + 4 <= 0) continue;
        const long o = base + c;
        if (c >= 0 && c + 3 < r) {
            float4 a = *(float4*)(p + o), b = *(float4*)(m + o), e = *(float4*)(v + o);
            a.x += 1; b.y += 1; e.z += 1;
            *(float4*)(p + o) = a; *(float4*)(m + o) = b; *(float4*)(v + o) = e;
        } else {
            for (int i = 0; i < 4; ++i)
                if (c + i >= 0 && c + i < r) { p[o + i] += 1; m[o + i] += 1; v[o + i] += 1; }
        }
    }
}
// wide pieces: 16 rows x 256 columns per WG, each wave instruction = one
// row's 1 KB run
__global__ __launch_bounds__(256) void wtiles(const Tile* t, float* p, float* m, float* v, int n) {
    const Tile tt = t[blockIdx.x];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int j = 0; j < 4; ++j) {
        const int r = tt.r0 + w + 4 * j;
        const int c = tt.c0 + 4 * lane;
        if (r >= n - 1 || c >= r) continue;
        const long o = (long)r * (r - 1) / 2 + c;
        if (c + 3 < r) {
            float4 a = *(float4*)(p + o), b = *(float4*)(m + o), e = *(float4*)(v + o);
            a.x += 1; b.y += 1; e.z += 1;
            *(float4*)(p + o) = a; *(float4*)(m + o) = b; *(float4*)(v + o) = e;
        } else {
            for (int i = 0; c + i < r; ++i) { p[o + i] += 1; m[o + i] += 1; v[o + i] += 1; }
        }
    }
}
// one-shot contiguous pieces: WG b handles floats [b*4096, (b+1)*4096) of each
// array once (tile-sized work units over contiguous memory)
__global__ __launch_bounds__(256) void oneshot(float4* p, float4* m, float4* v, long n4) {
    const long base = (long)blockIdx.x * 1024;
    float4 a[4], b[4], d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const long i = base + threadIdx.x + 256 * j;
        if (i < n4) { a[j] = p[i]; b[j] = m[i]; d[j] = v[i]; }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const long i = base + threadIdx.x + 256 * j;
        if (i < n4) { a[j].x += 1; b[j].y += 1; d[j].z += 1; p[i] = a[j]; m[i] = b[j]; v[i] = d[j]; }
    }
}
// persistent: WG loops over tiles blockIdx.x, +gridDim.x, ... of a list
__global__ __launch_bounds__(256) void ptiles(const Tile* t, int nt, float* p, float* m, float* v, int n) {
    const int col4 = threadIdx.x & 15, srow = threadIdx.x >> 4;
    for (int k = blockIdx.x; k < nt; k += gridDim.x) {
        const Tile tt = t[k];
        for (int j = 0; j < 4; ++j) {
            const int r = tt.r0 + srow + 16 * j;
            const int c = tt.c0 + 4 * col4;
            if (r >= n - 1 || c >= r) continue;
            const long o = (long)r * (r - 1) / 2 + c;
            if (c + 3 < r) {
                float4 a = *(float4*)(p + o), b = *(float4*)(m + o), d = *(float4*)(v + o);
                a.x += 1; b.y += 1; d.z += 1;
                *(float4*)(p + o) = a; *(float4*)(m + o) = b; *(float4*)(v + o) = d;
            } else {
                for (int i = 0; c + i < r; ++i) { p[o + i] += 1; m[o + i] += 1; v[o + i] += 1; }
            }
        }
    }
}
struct Sweep { int r0, c0, c1; };
__global__ __launch_bounds__(256) void sweep(const Sweep* t, float* p, float* m, float* v, int n) {
    const Sweep tt = t[blockIdx.x];
    const int col4 = threadIdx.x & 15, srow = threadIdx.x >> 4;
    for (int cb = tt.c0; cb < tt.c1; cb += 64) {
        for (int j = 0; j < 4; ++j) {
            const int r = tt.r0 + srow + 16 * j;
            const int c = cb + 4 * col4;
            if (r >= n - 1 || c >= r) continue;
            const long o = (long)r * (r - 1) / 2 + c;
            if (c + 3 < r) {
                float4 a = *(float4*)(p + o), b = *(float4*)(m + o), d = *(float4*)(v + o);
                a.x += 1; b.y += 1; d.z += 1;
                *(float4*)(p + o) = a; *(float4*)(m + o) = b; *(float4*)(v + o) = d;
            } else {
                for (int i = 0; c + i < r; ++i) { p[o + i] += 1; m[o + i] += 1; v[o + i] += 1; }
            }
        }
    }
}
__global__ __launch_bounds__(256) void stream(float4* p, float4* m, float4* v, long n4) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        float4 a = p[i], b = m[i], d = v[i];
        a.x += 1; b.y += 1; d.z += 1;
        p[i] = a; m[i] = b; v[i] = d;
    }
}
int main() {
    const int ns[3] = {2600, 1640, 82};
    // one layer at a time: n = 2600 (the big one, 3.37 M corr)
    const int n = 2600;
    const long nc = (long)(n - 1) * (n - 2) / 2;
    float *p, *m, *v;
    (void)hipMalloc(&p, (nc + 64) * 4); (void)hipMalloc(&m, (nc + 64) * 4); (void)hipMalloc(&v, (nc + 64) * 4);
    (void)hipMemset(p, 0, nc * 4); (void)hipMemset(m, 0, nc * 4); (void)hipMemset(v, 0, nc * 4);
    std::vector<Tile> ts;
    for (int r0 = 0; r0 < n - 1; r0 += 64)
        for (int c0 = 0; c0 < r0 + 63 && c0 < n - 2; c0 += 64) ts.push_back({r0, c0});
    Tile* dt; (void)hipMalloc(&dt, ts.size() * sizeof(Tile));
    (void)hipMemcpy(dt, ts.data(), ts.size() * sizeof(Tile), hipMemcpyHostToDevice);
    // XCD-aware order: tile i of band b goes to XCD (b % 8), consecutive in time
    std::vector<std::vector<Tile>> q(8);
    for (const Tile& t : ts) q[(t.r0 / 64) % 8].push_back(t);
    std::vector<Tile> tx;
    size_t len = 0;
    for (auto& x : q) len = std::max(len, x.size());
    for (size_t j = 0; j < len; ++j)
        for (int x = 0; x < 8; ++x) tx.push_back(j < q[x].size() ? q[x][j] : Tile{1 << 20, 0});
    Tile* dtx; (void)hipMalloc(&dtx, tx.size() * sizeof(Tile));
    (void)hipMemcpy(dtx, tx.data(), tx.size() * sizeof(Tile), hipMemcpyHostToDevice);
    auto make_sweeps = [&](int CH, bool xcd) {
        std::vector<std::vector<Sweep>> qq(xcd ? 8 : 1);
        int band = 0;
        for (int r0 = 0; r0 < n - 1; r0 += 64, ++band) {
            const int cmax = std::min(r0 + 64, n - 2);
            for (int c0 = 0; c0 < cmax; c0 += 64 * CH)
                qq[xcd ? band % 8 : 0].push_back({r0, c0, std::min(c0 + 64 * CH, cmax)});
        }
        std::vector<Sweep> out;
        size_t L = 0;
        for (auto& x : qq) L = std::max(L, x.size());
        for (size_t j = 0; j < L; ++j)
            for (auto& x : qq) out.push_back(j < x.size() ? x[j] : Sweep{1 << 20, 0, 0});
        Sweep* d; (void)hipMalloc(&d, out.size() * sizeof(Sweep));
        (void)hipMemcpy(d, out.data(), out.size() * sizeof(Sweep), hipMemcpyHostToDevice);
        return std::make_pair(d, (int)out.size());
    };
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float ms;
    const double bytes = 6.0 * nc * 4;
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(tiles, dim3(ts.size()), dim3(256), 0, 0, dt, p, m, v, n);
        hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
        printf("tile pattern  (%zu tiles): %7.2f us  %6.0f GB/s\n", ts.size(), ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
        hipEventRecord(a);
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(tiles, dim3(tx.size()), dim3(256), 0, 0, dtx, p, m, v, n);
        hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
        printf("tile pattern, XCD-grouped bands: %7.2f us  %6.0f GB/s\n", ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
        {
            // aligned tiles need one extra column block per band (windows shift left by < 32)
            std::vector<std::vector<Tile>> qa(8);
            int band = 0;
            for (int r0 = 0; r0 < n - 1; r0 += 64, ++band)
                for (int c0 = 0; c0 < std::min(r0 + 64, n - 2) + 32; c0 += 64) qa[band % 8].push_back({r0, c0});
            std::vector<Tile> ta;
            size_t L = 0;
            for (auto& x : qa) L = std::max(L, x.size());
            for (size_t j = 0; j < L; ++j)
                for (auto& x : qa) ta.push_back(j < x.size() ? x[j] : Tile{1 << 20, 0});
            Tile* dta; (void)hipMalloc(&dta, ta.size() * sizeof(Tile));
            (void)hipMemcpy(dta, ta.data(), ta.size() * sizeof(Tile), hipMemcpyHostToDevice);
            hipEventRecord(a);
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(atiles, dim3(ta.size()), dim3(256), 0, 0, dta, p, m, v, n);
            hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
            printf("ALIGNED windows, XCD-grouped (%zu WGs): %7.2f us  %6.0f GB/s\n", ta.size(), ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
        }
        for (int xcd = 0; xcd < 2; ++xcd) {
            std::vector<std::vector<Tile>> qa(xcd ? 8 : 1);
            int band = 0;
            for (int r0 = 0; r0 < n - 1; r0 += 16, ++band)
                for (int c0 = 0; c0 < std::min(r0 + 16, n - 2); c0 += 256) qa[xcd ? (band / 4) % 8 : 0].push_back({r0, c0});
            std::vector<Tile> ta;
            size_t L = 0;
            for (auto& x : qa) L = std::max(L, x.size());
            for (size_t j = 0; j < L; ++j)
                for (auto& x : qa) ta.push_back(j < x.size() ? x[j] : Tile{1 << 20, 0});
            Tile* dta; (void)hipMalloc(&dta, ta.size() * sizeof(Tile));
            (void)hipMemcpy(dta, ta.data(), ta.size() * sizeof(Tile), hipMemcpyHostToDevice);
            hipEventRecord(a);
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(wtiles, dim3(ta.size()), dim3(256), 0, 0, dta, p, m, v, n);
            hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
            printf("16x256 tiles, 1KB row runs, xcd=%d (%zu WGs): %7.2f us  %6.0f GB/s\n", xcd, ta.size(), ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
        }
        {
            const int nb = (int)((nc / 4 + 1023) / 1024);
            hipEventRecord(a);
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(oneshot, dim3(nb), dim3(256), 0, 0, (float4*)p, (float4*)m, (float4*)v, nc / 4);
            hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
            printf("one-shot contiguous 16KB pieces (%d WGs): %7.2f us  %6.0f GB/s\n", nb, ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
        }
        for (int grid : {256, 512, 768, 1024}) {
            hipEventRecord(a);
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(ptiles, dim3(grid), dim3(256), 0, 0, dt, (int)ts.size(), p, m, v, n);
            hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
            printf("persistent tiles grid %4d (band order):  %7.2f us  %6.0f GB/s\n", grid, ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
        }
        for (int CH : {1})
            for (int xcd = 0; xcd < 2; ++xcd) {
                auto sw = make_sweeps(CH, xcd);
                hipEventRecord(a);
                for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(sweep, dim3(sw.second), dim3(256), 0, 0, sw.first, p, m, v, n);
                hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
                printf("sweeps CH=%d xcd=%d (%d WGs): %7.2f us  %6.0f GB/s\n", CH, xcd, sw.second, ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
            }
        for (int grid : {512, 2048}) {
            hipEventRecord(a);
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(stream, dim3(grid), dim3(256), 0, 0, (float4*)p, (float4*)m, (float4*)v, nc / 4);
            hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
            printf("contiguous (grid %4d):      %7.2f us  %6.0f GB/s\n", grid, ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e9);
        }
    }
    (void)ns;
    return 0;
}
