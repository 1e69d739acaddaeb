// The frame the reference application presents per redraw -- State::render (src/state.rs:270-286):
// Scene::render into the two Bgra8UnormSrgb targets (src/scene.rs:470-522), then Bloom::render from them to
// the surface (src/bloom.rs:53-71) -- as one pipelined path on one GPU (include/bh_render.h, bh_presenter).
//
// The march is VALU-bound and ends in a serial tail (the few rays that run to the cap, one wave each), the
// bloom is latency-bound (LDS / load round trips, VALU 0.2-0.3 busy).  Run back to back on one stream they
// add; here frame i's bloom runs on a second stream while frame i + 1 marches, so it fills the CUs the
// march's tail leaves idle.  The presenter owns `depth` banks of `batch` (col, blackout) target pairs and
// `march_streams` march streams: call c marches its frames into bank c % depth (one bh_render_frames launch) on
// march stream c % march_streams, so with two the next call's march also starts under this call's serial tail
// (each stream keeps its own temporal order state); a bank is reused once its blooms have run (an event), and
// the caller's stream waits for the call's last bloom, so work the caller queues after bh_present sees the
// finished surfaces.  (The device has few hardware queues -- GPU_MAX_HW_QUEUES, 4 by default -- and streams
// beyond them share one, in order: so the presenter keeps to three streams at most.)
// Each surface equals the serial bh_render + bh_bloom bytes: the same kernels on the same inputs, only
// their streams differ (tests/test_gpu_present.py).
//
// Streams: by default both share every CU; the bloom's stream has the device's highest priority, so its
// workgroups are dispatched first as the march's waves retire.  bloom_cus > 0 splits the CUs instead
// (hipExtStreamCreateWithCUMask): the bloom on bloom_cus CUs spread over the mask (every n_cu / bloom_cus-th
// bit, so over every XCD whatever the bit -> XCD mapping), the march on the others.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <vector>

#include "bh_common.hpp"

struct bh_presenter {
    bh_ctx* ctx = nullptr;
    bh_presenter_desc d{};
    int device = 0;
    uint32_t depth = 2, n_march = 1;
    hipStream_t march[BH_PRESENT_DEPTH_MAX] = {}, bloom = nullptr;
    uint8_t* targets = nullptr;   // depth banks x batch x (col, blackout), width x height x 4 B each
    hipEvent_t bank_free[BH_PRESENT_DEPTH_MAX] = {};  // the bank's last blooms have run (never recorded: free)
    hipEvent_t marched[BH_PRESENT_DEPTH_MAX] = {};    // the bank's march has run
    hipEvent_t caller = nullptr;   // the caller's stream at the call (the surfaces' previous users)
    uint32_t call = 0;             // calls so far: the next call's bank and march stream are call % depth
    std::vector<bh_render_desc> descs;
};

namespace {

struct PresentDevice {  // the presenter's device current for the call, the caller's restored after it
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit PresentDevice(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) err = hipSetDevice(device);
    }
    ~PresentDevice() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int present_fail(hipError_t e, const char* what) {
    bh_set_last_error(std::string(what) + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? BH_ERR_OUT_OF_MEMORY : BH_ERR_HIP;
}

void destroy_parts(bh_presenter* p) {
    for (hipStream_t m : p->march)
        if (m) (void)hipStreamSynchronize(m);  // (null entries: the march streams past n_march)
    if (p->bloom) (void)hipStreamSynchronize(p->bloom);
    for (uint32_t k = 0; k < BH_PRESENT_DEPTH_MAX; ++k) {
        if (p->bank_free[k]) (void)hipEventDestroy(p->bank_free[k]);
        if (p->marched[k]) (void)hipEventDestroy(p->marched[k]);
        if (p->march[k]) (void)hipStreamDestroy(p->march[k]);
    }
    if (p->caller) (void)hipEventDestroy(p->caller);
    if (p->bloom) (void)hipStreamDestroy(p->bloom);
    if (p->targets) (void)hipFree(p->targets);
}

}  // namespace

extern "C" {

int bh_presenter_create(bh_ctx* ctx, const bh_presenter_desc* desc, bh_presenter** out) {
    if (!out) return bh_bad_arg(__func__, __LINE__);
    *out = nullptr;
    if (!ctx || !desc || desc->width == 0 || desc->height == 0 || desc->width > 65536u || desc->height > 65536u ||
        desc->max_iters == 0 || desc->max_iters > 65535u || desc->levels < 1 || desc->levels > 12 || desc->batch < 1 ||
        desc->batch > BH_PRESENT_BATCH_MAX || desc->math > BH_MATH_FAST || (desc->scene_flags & ~BH_SCENE_DEFAULT) != 0u ||
        desc->depth == 1u || desc->depth > BH_PRESENT_DEPTH_MAX || desc->march_streams > 2u ||
        desc->march_streams > (desc->depth ? desc->depth : 3u))
        return bh_bad_arg(__func__, __LINE__);
    const int device = bh_ctx_device(ctx);
    PresentDevice dev(device);
    if (dev.err != hipSuccess) return present_fail(dev.err, "hipSetDevice");
    int n_cu = 0;
    hipError_t e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return present_fail(e, "hipDeviceGetAttribute(CU count)");
    if (desc->bloom_cus >= (uint32_t)n_cu) return bh_bad_arg(__func__, __LINE__);  // the march keeps some CUs
    auto* p = new (std::nothrow) bh_presenter;
    if (!p) return BH_ERR_OUT_OF_MEMORY;
    p->ctx = ctx;
    p->d = *desc;
    p->device = device;
    p->depth = desc->depth ? desc->depth : 3u;
    // auto: a second march stream only for frames whose march leaves the GPU idle for most of its time (at most
    // 64 tiles per CU: 1280x720 one frame per call 0.280 -> 0.218 ms per presented frame; 1920x1080 0.316 ->
    // 0.375 and 4096x2048 0.779 -> 0.871 ms with two -- the extra stream then shares a hardware queue,
    // tools/bench_frame.py, profiles/r06/frame/)
    const uint64_t tiles = (uint64_t)((desc->width + 7u) / 8u) * ((desc->height + 7u) / 8u) * desc->batch;
    p->n_march = desc->march_streams ? desc->march_streams : (tiles <= 64ull * (uint64_t)n_cu ? 2u : 1u);
    const size_t img = (size_t)desc->width * desc->height * 4u;
    e = hipMalloc(&p->targets, (size_t)p->depth * desc->batch * 2u * img);
    if (e == hipSuccess && desc->bloom_cus > 0) {
        const uint32_t words = ((uint32_t)n_cu + 31u) / 32u, nb = desc->bloom_cus, step = (uint32_t)n_cu / nb;
        std::vector<uint32_t> bm(words, 0u), mm(words, 0u);
        for (uint32_t i = 0; i < nb; ++i) bm[(i * step) / 32u] |= 1u << ((i * step) % 32u);
        for (uint32_t c = 0; c < (uint32_t)n_cu; ++c)
            if (!(bm[c / 32u] & (1u << (c % 32u)))) mm[c / 32u] |= 1u << (c % 32u);
        for (uint32_t k = 0; k < p->n_march && e == hipSuccess; ++k)
            e = hipExtStreamCreateWithCUMask(&p->march[k], words, mm.data());
        if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&p->bloom, words, bm.data());
    } else if (e == hipSuccess) {
        int least = 0, greatest = 0;
        e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        (void)least;  // the march streams at the default priority, the bloom's above it
        for (uint32_t k = 0; k < p->n_march && e == hipSuccess; ++k)
            e = hipStreamCreateWithPriority(&p->march[k], hipStreamNonBlocking, 0);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&p->bloom, hipStreamNonBlocking, greatest);
    }
    for (uint32_t k = 0; k < p->depth && e == hipSuccess; ++k) {
        e = hipEventCreateWithFlags(&p->bank_free[k], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->marched[k], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->caller, hipEventDisableTiming);
    if (e != hipSuccess) {
        destroy_parts(p);
        delete p;
        return present_fail(e, "bh_presenter_create");
    }
    p->descs.resize(desc->batch);
    for (uint32_t i = 0; i < desc->batch; ++i) {
        bh_render_desc& r = p->descs[i];
        std::memset(&r, 0, sizeof r);
        r.width = desc->width;
        r.height = desc->height;
        r.max_iters = desc->max_iters;
        r.scene_flags = desc->scene_flags;
        r.format = BH_OUT_BGRA8_SRGB;
        r.math = desc->math;
        r.layout = BH_LAYOUT_ROWMAJOR;
        r.shard_index = 0;
        r.shard_count = 1;
        r.schedule = BH_SCHED_TILE;
    }
    *out = p;
    return BH_OK;
}

int bh_presenter_destroy(bh_presenter* p) {
    if (!p) return bh_bad_arg(__func__, __LINE__);
    {
        PresentDevice dev(p->device);
        destroy_parts(p);
    }
    delete p;
    return BH_OK;
}

int bh_present_frames(bh_presenter* p, uint32_t n, const bh_camera_uniform* cameras, const bh_uniforms* uniforms,
                      void* const* out_surfaces, void* hip_stream) {
    if (!p || !cameras || !uniforms || !out_surfaces || n < 1 || n > p->d.batch) return bh_bad_arg(__func__, __LINE__);
    for (uint32_t i = 0; i < n; ++i)
        if (!out_surfaces[i]) return bh_bad_arg(__func__, __LINE__);
    PresentDevice dev(p->device);
    if (dev.err != hipSuccess) return present_fail(dev.err, "hipSetDevice");
    hipStream_t caller = reinterpret_cast<hipStream_t>(hip_stream);
    const uint32_t bank = p->call % p->depth;
    // A call of 4 or more frames marches them in one launch whose frames overlap each other's tails and fill the
    // GPU: its blooms then gain nothing from a second stream (1920x1080, 16 frames per call: serial 0.279,
    // pipelined 0.296 ms per frame), so march and blooms run on the caller's stream, in order, with no
    // cross-stream handshake at all.
    const bool serial = n >= 4u;
    hipStream_t march = serial ? caller : p->march[p->call % p->n_march];
    const size_t img = (size_t)p->d.width * p->d.height * 4u;
    uint8_t* base = p->targets + (size_t)bank * p->d.batch * 2u * img;
    for (uint32_t i = 0; i < n; ++i) {
        p->descs[i].out_col = base + (2u * i) * img;
        p->descs[i].out_blackout = base + (2u * i + 1u) * img;
    }
    // the bank is free once the blooms of the call `depth` before have read it
    hipError_t e = hipStreamWaitEvent(march, p->bank_free[bank], 0);
    if (e != hipSuccess) return present_fail(e, "hipStreamWaitEvent(bank)");
    int st = bh_render_frames(p->ctx, n, cameras, uniforms, p->descs.data(), march);
    if (st != BH_OK) return st;
    if ((e = hipEventRecord(p->marched[bank], march)) != hipSuccess) return present_fail(e, "hipEventRecord(march)");
    hipStream_t bs = serial ? caller : p->bloom;
    // the surfaces: written after the caller's earlier work on them (its stream at this call), and after the
    // previous call's blooms (the ctx's bloom scratch is shared: never two chains at once)
    if (!serial) {
        if ((e = hipEventRecord(p->caller, caller)) != hipSuccess) return present_fail(e, "hipEventRecord(caller)");
        if ((e = hipStreamWaitEvent(bs, p->caller, 0)) != hipSuccess) return present_fail(e, "hipStreamWaitEvent(caller)");
    }
    if (p->call > 0 && (e = hipStreamWaitEvent(bs, p->bank_free[(p->call - 1u) % p->depth], 0)) != hipSuccess)
        return present_fail(e, "hipStreamWaitEvent(previous blooms)");
    if (bs != march && (e = hipStreamWaitEvent(bs, p->marched[bank], 0)) != hipSuccess)
        return present_fail(e, "hipStreamWaitEvent(march)");
    for (uint32_t i = 0; i < n; ++i) {
        st = bh_bloom(p->ctx, p->descs[i].out_col, p->descs[i].out_blackout, p->d.width, p->d.height, p->d.levels,
                      BH_BLOOM_AUTO, out_surfaces[i], bs);
        if (st != BH_OK) return st;
    }
    if ((e = hipEventRecord(p->bank_free[bank], bs)) != hipSuccess) return present_fail(e, "hipEventRecord(bloom)");
    // the caller's later work sees the finished surfaces
    if (!serial && (e = hipStreamWaitEvent(caller, p->bank_free[bank], 0)) != hipSuccess)
        return present_fail(e, "hipStreamWaitEvent(caller)");
    ++p->call;
    return BH_OK;
}

int bh_present(bh_presenter* p, const bh_camera_uniform* camera, const bh_uniforms* uniforms, void* out_surface,
               void* hip_stream) {
    void* const outs[1] = {out_surface};
    return bh_present_frames(p, 1, camera, uniforms, outs, hip_stream);
}

}  // extern "C"
