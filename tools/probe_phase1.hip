// Probe (tools/, not product code): the score-only DP of two adapters per lane in 16-bit halves,
// on the headline's cross-mode shape (391 tiles of 256 windows x 23 adapter pairs, 150 columns,
// 24 rows), in three forms:
//   pk     v2 = int16 x 2 vector ops: the compiler's v_pk_add_u16 / v_pk_max_i16 (sf::filter_lane)
//   swar   the adds as ONE 32-bit v_add_u32 over both halves (values biased by 0x4000 per half, so
//          no half ever carries into the other), the maxes as v_pk_max_u16 on the biased halves
//   swar_bj  swar plus the last-row scout's first-maximum column per half (what a score phase of
//          a two-phase end-trim core must hand the attribute phase)
// Every form's result is checked against a scalar host DP on the first windows. Timed with events,
// clock from s_memtime / s_memrealtime per wave as tools/replay_k24.hip.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/probe_phase1 tools/probe_phase1.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

constexpr int RPL = 24, N = 150, TILES = 391, PAIRS = 23, NQ = N / 4 + 3;
constexpr int MA = 3, MI = -6, GO = -5, GE = -2;
constexpr int BIAS = 0x4000;

typedef int16_t v2 __attribute__((ext_vector_type(2)));
typedef uint16_t u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pkmaxu(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u2, a), __builtin_bit_cast(u2, b)));
}

struct Reader {
    const uint32_t *q;
    uint32_t lo, hi, nx;
    __device__ Reader(const uint32_t *b) : q(b) { lo = q[0]; hi = q[256]; nx = q[512]; }
    __device__ __forceinline__ int operator()(int j) {
        const int k = j - 1;
        if (k > 0 && (k & 3) == 0) { lo = hi; hi = nx; nx = q[(k / 4 + 2) * 256]; }
        return (int)(((((uint64_t)hi << 32) | lo) >> (8 * (k & 3))) & 0xFFu);
    }
};

// tab[pair][code][slot]: (adapter A, adapter B) substitution minus gap open, packed per form
template <int FORM>
__global__ __launch_bounds__(256) void k_probe(const uint32_t *tiles, const uint32_t *tabs, int32_t *out,
                                               unsigned long long *clk) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[8 * RPL];
    const int b = blockIdx.x, pr = b % PAIRS, tile = b / PAIRS;
    for (int e = threadIdx.x; e < 8 * RPL; e += 256) tab[e] = tabs[pr * 8 * RPL + e];
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    Reader rd(tiles + (size_t)tile * NQ * 256 + threadIdx.x);
    int32_t res = 0, resj = 0;
    if (FORM == 0) {
        const v2 go2 = {(int16_t)GO, (int16_t)GO}, ge2 = {(int16_t)GE, (int16_t)GE};
        const v2 neg = {-8192, -8192};
        v2 G[RPL + 1], H[RPL + 1];
#pragma unroll
        for (int s = 1; s <= RPL; ++s) { G[s] = go2; H[s] = neg; }
        v2 best = {0, 0};
        int r = rd(1);
#pragma unroll 1
        for (int j = 1; j <= N; ++j) {
            const int rn = j < N ? rd(j + 1) : 0;
            const v2 *t = reinterpret_cast<const v2 *>(tab + r * RPL) - 1;
            v2 gup = go2, vup = neg, diag = go2 + t[1];
#pragma unroll
            for (int s = 1; s <= RPL; ++s) {
                v2 dnx = diag;
                if (s < RPL) dnx = G[s] + t[s + 1];
                const v2 hn = __builtin_elementwise_max(H[s] + ge2, G[s]);
                const v2 vn = __builtin_elementwise_max(vup + ge2, gup);
                const v2 sn = __builtin_elementwise_max(__builtin_elementwise_max(diag, vn), hn);
                G[s] = sn + go2;
                H[s] = hn;
                gup = G[s];
                vup = vn;
                diag = dnx;
            }
            best = __builtin_elementwise_max(best, G[RPL] - go2);
            r = rn;
        }
        res = (int32_t)__builtin_bit_cast(uint32_t, best);
    } else {
        // biased halves (x + BIAS each); a per-half constant c is added as the signed 32-bit word
        // c + c * 2^16: lo' = x_lo + c without a borrow (biased values stay >= |c|), hi' = x_hi + c
        const uint32_t c_go = (uint32_t)(GO + GO * 65536), c_ge = (uint32_t)(GE + GE * 65536);
        const uint32_t bias2 = (uint32_t)BIAS * 0x10001u;
        const uint32_t neg = bias2 - 8192u * 0x10001u;
        uint32_t G[RPL + 1], H[RPL + 1];
#pragma unroll
        for (int s = 1; s <= RPL; ++s) { G[s] = bias2 + c_go; H[s] = neg; }
        uint32_t best = bias2;
        int bjA = 0, bjB = 0;
        int r = rd(1);
#pragma unroll 1
        for (int j = 1; j <= N; ++j) {
            const int rn = j < N ? rd(j + 1) : 0;
            const uint32_t *t = tab + r * RPL - 1;
            uint32_t gup = bias2 + c_go, vup = neg, diag = bias2 + c_go + t[1];
#pragma unroll
            for (int s = 1; s <= RPL; ++s) {
                uint32_t dnx = diag;
                if (s < RPL) dnx = G[s] + t[s + 1];
                const uint32_t hn = pkmaxu(H[s] + c_ge, G[s]);
                const uint32_t vn = pkmaxu(vup + c_ge, gup);
                const uint32_t sn = pkmaxu(pkmaxu(diag, vn), hn);
                G[s] = sn + c_go;
                H[s] = hn;
                gup = G[s];
                vup = vn;
                diag = dnx;
            }
            const uint32_t last = G[RPL] - c_go;
            if (FORM == 2 && j < N) {
                // first maximum per half (strict >)
                const uint32_t nb = pkmaxu(best, last);
                bjA = ((nb ^ best) & 0xFFFFu) ? j : bjA;
                bjB = ((nb ^ best) >> 16) ? j : bjB;
                best = nb;
            } else {
                best = pkmaxu(best, last);
            }
            r = rn;
        }
        res = (int32_t)(best - bias2);
        resj = bjA | (bjB << 16);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = r1 - r0;
    }
    const size_t o = ((size_t)pr * TILES * 256 + (size_t)tile * 256 + threadIdx.x) * 2;
    out[o] = res;
    out[o + 1] = resj;
}

// host reference: best score over the last row (the probe's scout), S(i, 0) = S(0, j) = 0
static int host_best(const uint8_t *w, const uint8_t *a, int L) {
    const int NEGI = -100000;
    std::vector<int> S((size_t)(L + 1) * (N + 1)), V(S.size()), Hh(S.size());
    auto at = [&](int i, int j) { return (size_t)i * (N + 1) + j; };
    for (int j = 0; j <= N; ++j) { S[at(0, j)] = 0; V[at(0, j)] = NEGI; Hh[at(0, j)] = NEGI; }
    for (int i = 1; i <= L; ++i) { S[at(i, 0)] = 0; Hh[at(i, 0)] = NEGI; V[at(i, 0)] = NEGI; }
    for (int i = 1; i <= L; ++i)
        for (int j = 1; j <= N; ++j) {
            Hh[at(i, j)] = std::max(Hh[at(i, j - 1)] + GE, S[at(i, j - 1)] + GO);
            V[at(i, j)] = std::max(V[at(i - 1, j)] + GE, S[at(i - 1, j)] + GO);
            const int d = S[at(i - 1, j - 1)] + (a[i - 1] == w[j - 1] ? MA : MI);
            S[at(i, j)] = std::max(d, std::max(Hh[at(i, j)], V[at(i, j)]));
        }
    int best = 0;
    for (int j = 1; j <= N; ++j) best = std::max(best, S[at(L, j)]);
    return best;
}

static double eff_clock(const unsigned long long *d_clk, size_t waves) {
    std::vector<unsigned long long> h(2 * waves);
    CHECK(hipMemcpy(h.data(), d_clk, h.size() * 8, hipMemcpyDeviceToHost));
    double t = 0, r = 0;
    for (size_t w = 0; w < waves; ++w) { t += (double)h[2 * w]; r += (double)h[2 * w + 1]; }
    return r > 0 ? t / r * 0.1 : 0.0;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    uint32_t x = 777;
    auto rnd = [&]() { x = x * 1103515245u + 12345u; return (x >> 16) % 4u; };
    const int nw = TILES * 256;
    std::vector<uint8_t> win((size_t)nw * N);
    for (auto &c : win) c = (uint8_t)rnd();
    std::vector<uint8_t> adp((size_t)2 * PAIRS * RPL);
    for (auto &c : adp) c = (uint8_t)rnd();
    // plant adapter 0 into some windows
    for (int w = 0; w < nw; w += 7)
        for (int k = 0; k < RPL; ++k) win[(size_t)w * N + 60 + k] = adp[k];
    std::vector<uint32_t> tiles((size_t)TILES * NQ * 256, 0);
    for (int w = 0; w < nw; ++w)
        for (int j = 0; j < N; ++j)
            tiles[((size_t)(w / 256) * NQ + j / 4) * 256 + (w % 256)] |= (uint32_t)win[(size_t)w * N + j] << (8 * (j % 4));
    std::vector<uint32_t> tab_pk((size_t)PAIRS * 8 * RPL), tab_sw(tab_pk.size());
    for (int p = 0; p < PAIRS; ++p)
        for (int c = 0; c < 8; ++c)
            for (int s = 0; s < RPL; ++s) {
                const int va = (c == adp[(2 * p) * RPL + s] ? MA : MI) - GO;
                const int vb = (c == adp[(2 * p + 1) * RPL + s] ? MA : MI) - GO;
                tab_pk[((size_t)p * 8 + c) * RPL + s] = (uint32_t)(uint16_t)(int16_t)va | ((uint32_t)(uint16_t)(int16_t)vb << 16);
                tab_sw[((size_t)p * 8 + c) * RPL + s] = (uint32_t)(va + vb * 65536);
            }
    uint32_t *d_tiles, *d_pk, *d_sw;
    int32_t *d_out;
    unsigned long long *d_clk;
    const int blocks = TILES * PAIRS;
    CHECK(hipMalloc(&d_tiles, tiles.size() * 4));
    CHECK(hipMalloc(&d_pk, tab_pk.size() * 4));
    CHECK(hipMalloc(&d_sw, tab_sw.size() * 4));
    CHECK(hipMalloc(&d_out, (size_t)PAIRS * nw * 8));
    CHECK(hipMalloc(&d_clk, (size_t)blocks * 4 * 16));
    CHECK(hipMemcpy(d_tiles, tiles.data(), tiles.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_pk, tab_pk.data(), tab_pk.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_sw, tab_sw.data(), tab_sw.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char *names[] = {"pk", "swar", "swar_bj"};
    void (*ks[])(const uint32_t *, const uint32_t *, int32_t *, unsigned long long *) = {k_probe<0>, k_probe<1>, k_probe<2>};
    std::vector<int32_t> h_out((size_t)PAIRS * nw * 2);
    for (int f = 0; f < 3; ++f) {
        const uint32_t *tb = f == 0 ? d_pk : d_sw;
        auto launch = [&]() { hipLaunchKernelGGL(ks[f], dim3(blocks), dim3(256), 0, 0, d_tiles, tb, d_out, d_clk); };
        for (int w = 0; w < 3; ++w) launch();
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int k = 0; k < reps; ++k) launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        const double ghz = eff_clock(d_clk, (size_t)blocks * 4);
        CHECK(hipMemcpy(h_out.data(), d_out, h_out.size() * 4, hipMemcpyDeviceToHost));
        int bad = 0, checked = 0;
        for (int p = 0; p < 2 && p < PAIRS; ++p)
            for (int w = 0; w < 600; w += 3) {
                const int32_t v = h_out[((size_t)p * nw + w) * 2];
                const int a = (int)(int16_t)(v & 0xFFFF), b = (int)(int16_t)((uint32_t)v >> 16);
                const int ra = host_best(&win[(size_t)w * N], &adp[(2 * p) * RPL], RPL);
                const int rb = host_best(&win[(size_t)w * N], &adp[(2 * p + 1) * RPL], RPL);
                checked += 2;
                bad += (a != ra) + (b != rb);
            }
        const double cells = (double)blocks * 256 * 2 * RPL * N;
        std::printf("{\"form\": \"%s\", \"ms\": %.4f, \"clock_ghz\": %.4f, \"cells_per_s\": %.4e, "
                    "\"cycles_per_cell_per_simd\": %.3f, \"checked\": %d, \"mismatches\": %d}\n",
                    names[f], ms, ghz, cells / (ms * 1e-3), 1024.0 * ms * 1e-3 * ghz * 1e9 / (cells / 64.0), checked, bad);
        std::fflush(stdout);
    }
    return 0;
}
