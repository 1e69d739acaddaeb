// Host emulation of the final fix-up pass's global reads (bh_bloom.hip fixup_gather_kernel<EPI_FINAL> with its
// records and column strips) and of the quad pass's strip writes (up_sepq_kernel's STRIPS epilogue), for one
// frame size: every index each lane would form is checked against its buffer's size.  A debugging aid for a
// GPU memory fault -- it runs on the CPU from the same host plan builders the library uploads.
//   g++ -O1 -std=c++17 -c tools/bloom_fixup_addr.cpp -o /tmp/fa.o &&
//   hipcc --offload-arch=gfx950 /tmp/fa.o black_hole_ray_marching_amd/_build/bh_bloom.o -o /tmp/fa
//   /tmp/fa W H [W H ...]          or          /tmp/fa sweep N SEED MAXW MAXH
// Exit status 1 when any index leaves its buffer.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" bool bh_bloom_same_plan(uint32_t w, uint32_t h, uint32_t* outp);
extern "C" uint32_t bh_bloom_strip_table(uint32_t w, const uint32_t* list, uint32_t nc, uint32_t* stc);
extern "C" void bh_bloom_fixup_records(uint32_t w, uint32_t h, const uint32_t* plan, const uint32_t* list, uint32_t nc,
                                       uint32_t nr, uint32_t* out);

static uint64_t bad = 0;
static void check(const char* what, uint64_t idx, uint64_t n, uint64_t lane) {
    if (idx < n) return;
    if (bad++ < 12) std::printf("OOB %s: index %llu of %llu (lane %llu)\n", what, (unsigned long long)idx, (unsigned long long)n,
                                (unsigned long long)lane);
}

static uint64_t run(uint32_t W, uint32_t H, bool verbose) {
    bad = 0;
    std::vector<uint32_t> plan(2u * ((size_t)W + H));
    if (!bh_bloom_same_plan(W, H, plan.data())) { std::printf("no plan\n"); return 1; }
    std::vector<uint32_t> list;
    uint32_t nc = 0, nr = 0;
    for (uint32_t x = 0; x < W; ++x) if (plan[2u * x + 1u]) { list.push_back(x); ++nc; }
    for (uint32_t y = 0; y < H; ++y) if (plan[2u * ((size_t)W + y) + 1u]) { list.push_back(y); ++nr; }
    std::vector<uint32_t> rec(8u * (size_t)(nc + nr));
    bh_bloom_fixup_records(W, H, plan.data(), list.data(), nc, nr, rec.data());
    std::vector<uint32_t> stc(W);
    const uint32_t stw = nc ? bh_bloom_strip_table(W, list.data(), nc, stc.data()) : 0u;
    for (uint32_t k = 0; k < nc; ++k) rec[8u * k + 7u] = stc[list[k]];
    if (verbose) std::printf("%ux%u: %u inexact columns, %u rows, %u strip columns\n", W, H, nc, nr, stw);
    const uint64_t texel_n = (uint64_t)W * H, plan_n = 2u * ((uint64_t)W + H) / 2u, strip_n = 3ull * stw * H;
    auto P = [&](uint64_t i) { check("plan", i, plan_n, 0); return std::make_pair(plan[2u * i], plan[2u * i + 1u]); };
    // the quad pass's strip writes: pixel (x, y) with st = stc[x] != 0 writes strips[(st - 1) * H + y + k * stw * H]
    for (uint32_t x = 0; x < W; ++x)
        if (stc[x]) for (uint32_t y = 0; y < H; ++y) for (uint32_t k = 0; k < 3; ++k)
            check("strip write", (uint64_t)(stc[x] - 1u) * H + y + (uint64_t)k * stw * H, strip_n, x);
    // fixup_gather_kernel<EPI_FINAL>, rec != null, strips != null
    const uint64_t ncl = (uint64_t)nc * H, n = ncl + (uint64_t)nr * W, lanes = (n + 255u) / 256u * 256u;
    for (uint64_t i = 0; i < lanes; ++i) {
        uint32_t x = 0, y = 0, qx = 0, k = 0;
        bool live = true, col = true;
        std::pair<uint32_t, uint32_t> PX[3], PY[3], cx, cy;
        if (i < ncl) { k = (uint32_t)(i / H); y = (uint32_t)(i % H); }
        else {
            const uint64_t j = i - ncl;
            live = j < (uint64_t)nr * W;
            col = false;
            if (live) { k = nc + (uint32_t)(j / W); x = (uint32_t)(j % W); }
        }
        check("rec", 8ull * k + 7u, rec.size(), i);
        const uint32_t* r = rec.data() + 8u * k;
        const std::pair<uint32_t, uint32_t> e0{r[1], r[2]}, e1{r[3], r[4]}, e2{r[5], r[6]};
        if (col) {
            x = r[0]; qx = r[7] - 1u;
            PX[0] = e0; PX[1] = e1; PX[2] = e2;
            const uint32_t yc = y < H - 1u ? y : H - 1u;
            PY[1] = P(W + yc); PY[0] = P(W + (yc ? yc - 1u : 0u)); PY[2] = P(W + (yc + 1u < H ? yc + 1u : H - 1u));
        } else {
            y = r[0];
            PY[0] = e0; PY[1] = e1; PY[2] = e2;
            const uint32_t xc = x < W - 1u ? x : W - 1u;
            PX[1] = P(xc); PX[0] = P(xc ? xc - 1u : 0u); PX[2] = P(xc + 1u < W ? xc + 1u : W - 1u);
        }
        live = live && x < W && y < H;
        cx = PX[1]; cy = PY[1];
        if (!live) { x = y = 0; cx = P(0); cy = P(W); PX[0] = PX[1] = PX[2] = cx; PY[0] = PY[1] = PY[2] = cy; }
        if (i >= ncl && cx.second != 0u) live = false;
        const bool sl = i < ncl;
        // gather_img: at(x, r) = min(x - xb, xm) * cs + r * rs (+ image base)
        auto gather = [&](uint32_t im, std::pair<uint32_t, uint32_t> a, std::pair<uint32_t, uint32_t> b, const char* what) {
            const uint32_t x0 = a.first & 0xFFFFu, x1 = a.first >> 16, r0 = b.first & 0xFFFFu, r1 = b.first >> 16;
            const bool ex = a.second != 0u, ey = b.second != 0u;
            auto at = [&](uint32_t tx, uint32_t ty) -> uint64_t {
                if (sl) {
                    const uint32_t off = (uint32_t)((int32_t)tx - ((int32_t)x - (int32_t)qx));
                    return (uint64_t)im * stw * H + (uint64_t)(off < stw - 1u ? off : stw - 1u) * H + ty;
                }
                return (uint64_t)ty * W + tx;
            };
            const uint64_t lim = sl ? strip_n : texel_n;
            check(what, at(x0, r0), lim, i);
            if (ex) check(what, at(x1, r0), lim, i);
            if (ey) check(what, at(x0, r1), lim, i);
            if (ex && ey) check(what, at(x1, r1), lim, i);
        };
        gather(0u, cx, cy, "A");
        auto pick = [&](uint32_t u, uint32_t c, std::pair<uint32_t, uint32_t>* Q, uint32_t base) {
            if (u == c) return Q[1];
            if (u + 1u == c) return Q[0];
            if (u == c + 1u) return Q[2];
            return P(base + u);
        };
        const bool ex = cx.second != 0u, ey = cy.second != 0u;
        const auto px0 = pick(cx.first & 0xFFFFu, x, PX, 0u), px1 = pick(cx.first >> 16, x, PX, 0u);
        const auto py0 = pick(cy.first & 0xFFFFu, y, PY, W), py1 = pick(cy.first >> 16, y, PY, W);
        for (uint32_t im = 1; im <= 2; ++im) {
            gather(im, px0, py0, im == 1 ? "B" : "C");
            if (ex) gather(im, px1, py0, im == 1 ? "B" : "C");
            if (ey) gather(im, px0, py1, im == 1 ? "B" : "C");
            if (ex && ey) gather(im, px1, py1, im == 1 ? "B" : "C");
        }
        if (live) check("out", (uint64_t)y * W + x, texel_n, i);
    }
    if (verbose || bad)
        std::printf("%ux%u: %llu lanes, %llu out-of-range indices\n", W, H, (unsigned long long)lanes, (unsigned long long)bad);
    return bad;
}

int main(int argc, char** argv) {
    uint64_t total = 0;
    if (argc >= 6 && std::strcmp(argv[1], "sweep") == 0) {
        const uint32_t n = (uint32_t)std::atoi(argv[2]), mw = (uint32_t)std::atoi(argv[4]), mh = (uint32_t)std::atoi(argv[5]);
        uint64_t s = (uint64_t)std::atoll(argv[3]) * 0x9E3779B97F4A7C15ull + 1u;
        auto next = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t W = 1u + (uint32_t)(next() % mw), H = 1u + (uint32_t)(next() % mh);
            total += run(W, H, false) != 0;
        }
        std::printf("%u sizes, %llu with out-of-range indices\n", n, (unsigned long long)total);
    } else {
        for (int a = 1; a + 1 < argc; a += 2) total += run((uint32_t)std::atoi(argv[a]), (uint32_t)std::atoi(argv[a + 1]), true) != 0;
    }
    return total ? 1 : 0;
}
