// Where the waves of K1 pp's small-shard geometry land: every wave of a
// 4-wave workgroup grid (1024 workgroups, one resident round at 16 waves per
// CU) records its HW_ID (SIMD, CU, SH, SE, workgroup slot) and XCC_ID, and
// the host counts, per SIMD, the waves of each in-workgroup index. If wave 3
// (the short one of a 12.5k-row shard: 2, 2, 2, 1 words) always lands on one
// SIMD, that SIMD idles half the sweep.
// Build: hipcc --offload-arch=gfx950 -O3 -o hwid tools/ubench/hwid.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256) void k_hwid(uint32_t *out, uint32_t spin) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    // keep the waves resident together for a while (VALU work, no memory)
    float a = (float)threadIdx.x;
    for (uint32_t i = 0; i < spin; ++i) a = a * 0.999f + 1.0f;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t idx = blockIdx.x * (blockDim.x >> 6) + wv;
    if (lane == 0) {
        out[idx * 4 + 0] = hw;
        out[idx * 4 + 1] = xcc;
        out[idx * 4 + 2] = (uint32_t)a;
    }
}

int main() {
    const int blocks = 1024, waves = 4;
    uint32_t *d;
    hipMalloc(&d, blocks * waves * 16);
    hipLaunchKernelGGL(k_hwid, dim3(blocks), dim3(64 * waves), 0, 0, d, 20000u);
    hipDeviceSynchronize();
    std::vector<uint32_t> h(blocks * waves * 4);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13] tg[19:16]
    std::map<std::tuple<int, int, int, int>, std::vector<int>> cu_simd_w3;  // (xcc, se, sh, cu) -> simd hist of wv 3
    std::map<std::tuple<int, int, int, int>, int> cu_blocks;
    int per_simd_wv[4][4] = {};
    for (int b = 0; b < blocks; ++b)
        for (int w = 0; w < waves; ++w) {
            const uint32_t hw = h[(b * waves + w) * 4], xcc = h[(b * waves + w) * 4 + 1] & 0xF;
            const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7,
                      tg = (hw >> 16) & 15;
            per_simd_wv[w][simd]++;
            auto key = std::make_tuple((int)xcc, se, sh, cu);
            auto &v = cu_simd_w3[key];
            if (v.empty()) v.assign(4, 0);
            if (w == 3) v[simd]++;
            if (w == 0) cu_blocks[key]++;
            if (b < 24)
                printf("block %4d wave %d: xcc %u se %d sh %d cu %2d simd %d tg %2d waveslot %u\n", b, w, xcc, se, sh, cu,
                       simd, tg, hw & 15);
        }
    printf("waves by (in-workgroup index, SIMD):\n");
    for (int w = 0; w < waves; ++w)
        printf("  wv %d: %d %d %d %d\n", w, per_simd_wv[w][0], per_simd_wv[w][1], per_simd_wv[w][2], per_simd_wv[w][3]);
    int n = 0;
    for (auto &kv : cu_simd_w3) {
        if (n++ < 16)
            printf("cu (xcc %d se %d sh %d cu %d): %d blocks, wv3 per simd %d %d %d %d\n", std::get<0>(kv.first),
                   std::get<1>(kv.first), std::get<2>(kv.first), std::get<3>(kv.first), cu_blocks[kv.first], kv.second[0],
                   kv.second[1], kv.second[2], kv.second[3]);
    }
    printf("distinct CUs: %zu\n", cu_simd_w3.size());
    hipFree(d);
    return 0;
}
