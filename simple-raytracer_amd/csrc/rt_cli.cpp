// rt_cli.cpp -- drop-in replacement for the reference executable
// (`SimpleRayTracer <scene.txt>`, main.cpp:60-657): parses the scene, renders
// it on MI355X through the C ABI of rt_hip.h and writes <scene>.ppm in the
// reference's P3 format.  Messages and exit behaviour follow main():
//   no argument          -> stdout message, exit 0           (main.cpp:653)
//   unreadable file      -> stdout message, exit 0           (main.cpp:567)
//   missing command      -> stdout "Error: Requires ...", 0  (main.cpp:574-602)
//   bad command          -> std::cerr lines, uncaught exception (abort)
// New optional flags (the reference has none): --depth N, --imsize W H,
// --gpus N (rows dealt to N devices in 8-row blocks), --device D,
// --gather host|rccl (how the devices' rows come together; host, the default:
// each device copies its rows to the host; rccl: one RCCL gather to the first
// device over xGMI -- the writer's values as bytes, 3 B per pixel, or the
// floats when a value is outside 0..255 -- a device-side de-interleave and
// one copy to the host --
// opt-in until a multi-device node has run tests/test_gpu_parity.py::
// test_cli_rccl_gather_multi_device), --float-out FILE (raw float32 H*W*3
// framebuffer), --stats, --stats-json FILE (the one-shot run's phases on
// the host clock: parse, scene upload, BVH build, render, device->host copy,
// quantise + P3 write; '-' = stderr).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <iostream>
#include <stdexcept>
#include <string>
#include <thread>
#include <memory>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "rt_hip.h"
#include "rt_host.h"

namespace {

const int kRowBlock = 8;

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// The host image, uninitialised: every float is written by the device->host
// copies before it is read (zero-filling C5's 3.2 GB took 0.53 s, more than
// the copy itself)
struct HostImage {
    std::unique_ptr<float[]> p;
    size_t n;
    explicit HostImage(size_t count) : p(new float[count]), n(count) {}
    float *data() { return p.get(); }
    size_t size() const { return n; }
    float *begin() { return p.get(); }
};

// One device, P3 out: the image comes to the host in blocks of rows through
// two pinned buffers, and each block is formatted and written (rth_ppm_*)
// while the next one copies -- the copy (C5: 3.2 GB, 0.13-0.25 s) hides
// behind the writer (0.3 s).  Returns rth_ppm_close's result (0 or -1); a
// HIP error goes to hip_rc.
int stream_ppm(const char *path, const float *dimg, int W, int H, int &hip_rc) {
    const size_t row = (size_t)W * 3;
    int R = (int)std::max<size_t>(1, std::min<size_t>((size_t)H, (size_t(64) << 20) / (row * sizeof(float))));
    if (const char *e = std::getenv("RT_PPM_BLOCK_ROWS")) R = std::max(1, std::min(H, std::atoi(e)));   // test hook
    const int nb = (H + R - 1) / R;
    float *pin[2] = {nullptr, nullptr};
    hipStream_t cs = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    rth_ppm_stream *ps = nullptr;
    if (rth_ppm_open(path, W, H, 0, &ps) != 0) {
        if (ps) (void)rth_ppm_close(ps);
        return -1;
    }
    const size_t bytes = (size_t)R * row * sizeof(float);
    if (hipHostMalloc((void **)&pin[0], bytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&pin[1], bytes, hipHostMallocDefault) != hipSuccess ||
        hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&ev[0]) != hipSuccess ||
        hipEventCreate(&ev[1]) != hipSuccess)
        hip_rc = RT_E_HIP;
    auto rows_of = [&](int b) { return std::min(R, H - b * R); };
    auto issue = [&](int b) {
        if (hipMemcpyAsync(pin[b & 1], dimg + (size_t)b * R * row, (size_t)rows_of(b) * row * sizeof(float),
                           hipMemcpyDeviceToHost, cs) != hipSuccess ||
            hipEventRecord(ev[b & 1], cs) != hipSuccess)
            hip_rc = RT_E_HIP;
    };
    if (!hip_rc && nb > 0) issue(0);
    bool good = true;
    for (int b = 0; !hip_rc && b < nb; b++) {
        if (b + 1 < nb) issue(b + 1);              // into the buffer block b - 1 has left
        if (hip_rc || hipEventSynchronize(ev[b & 1]) != hipSuccess) {
            hip_rc = RT_E_HIP;
            break;
        }
        if (rth_ppm_write_rows(ps, pin[b & 1], rows_of(b)) != 0) good = false;
    }
    if (cs) (void)hipStreamSynchronize(cs);
    const int wr = rth_ppm_close(ps) == 0 && good ? 0 : -1;
    for (int k = 0; k < 2; k++) {
        if (pin[k]) (void)hipHostFree(pin[k]);
        if (ev[k]) (void)hipEventDestroy(ev[k]);
    }
    if (cs) (void)hipStreamDestroy(cs);
    return wr;
}

// One device, P3 out from the writer's pixel values as bytes: the device
// quantises the image (rt_quantize_u8, exact for values 0..255), 3 bytes per
// pixel cross PCIe instead of 12 (C3: 50 MB instead of 201 MB, ~5 ms instead
// of ~19 through pageable memory), and the writer formats the bytes
// (rth_ppm_write_rows_u8, in row blocks of RT_PPM_BLOCK_ROWS when set: a
// test hook).  Returns 1 when some value is not 0..255 (NaN, a background
// above 1: the floats must be written, nothing was written), else 0 on
// success or -1 on a write error; a HIP error goes to hip_rc.  d2h_ms: the
// copy's time.  (A copier thread overlapping the copy with the writer was
// slower on C3 and C5, profiles/r05/e2e_s2*.txt: the pageable copy's
// staging competes with the writer's threads for the lease's cores.)
int write_ppm_bytes(const char *path, const float *dimg, int W, int H, int &hip_rc, double &d2h_ms) {
    const size_t n = (size_t)W * H * 3, row = (size_t)W * 3;
    unsigned char *d8 = nullptr;
    unsigned *dflag = nullptr;
    unsigned flag = 0;
    if (hipMalloc((void **)&d8, std::max<size_t>(4, (n + 3) / 4 * 4)) != hipSuccess ||
        hipMalloc((void **)&dflag, sizeof(unsigned)) != hipSuccess ||
        hipMemset(dflag, 0, sizeof(unsigned)) != hipSuccess || rt_quantize_u8(dimg, (long long)n, d8, dflag, nullptr) ||
        hipMemcpy(&flag, dflag, sizeof flag, hipMemcpyDeviceToHost) != hipSuccess) {
        hip_rc = RT_E_HIP;
    }
    int ret = 0;
    if (!hip_rc && (flag & 1u)) ret = 1;
    if (!hip_rc && ret == 0) {
        std::unique_ptr<unsigned char[]> host(new unsigned char[n]);
        const auto t0 = Clock::now();
        if (hipMemcpy(host.get(), d8, n, hipMemcpyDeviceToHost) != hipSuccess) hip_rc = RT_E_HIP;
        d2h_ms = ms_since(t0);
        int R = H;
        if (const char *e = std::getenv("RT_PPM_BLOCK_ROWS")) R = std::max(1, std::min(H, std::atoi(e)));   // test hook
        rth_ppm_stream *ps = nullptr;
        bool good = !hip_rc && rth_ppm_open(path, W, H, 0, &ps) == 0;
        for (int y = 0; good && y < H; y += R)
            if (rth_ppm_write_rows_u8(ps, host.get() + (size_t)y * row, std::min(R, H - y)) != 0) good = false;
        if (ps && rth_ppm_close(ps) != 0) good = false;
        ret = good ? 0 : -1;
    }
    if (d8) (void)hipFree(d8);
    if (dflag) (void)hipFree(dflag);
    return ret;
}

// The kernel instantiation with counters (rays by kind, executed tests)
// only when the run reports them (--stats, --stats-json): ~4 % slower
void set_counters(rt_scene *s, bool on) { (void)rt_scene_set_option(s, "counters", on ? 1 : 0); }
bool g_counters = false;

// One process, N devices: every device renders its row set (rth_row_set)
// into HBM, one RCCL gather collects the N buffers on the first device, a
// device-side de-interleave puts the rows in image order, one copy brings the
// image to the host.  The seam is the reference's single render call
// (main.cpp:607), its row loop (main.cpp:718) split across the devices.
//
// What crosses xGMI is the P3 writer's pixel values as bytes (3 B per pixel,
// rt_quantize_u8 on each device; bench.py's gather does the same): a quarter
// of the floats' bytes (C5 at N = 8: 101 MB per rank instead of 403).  When
// some device flags a value outside 0..255 (NaN, a background above 1), or
// the floats are wanted (want_floats: --float-out), the floats are gathered
// instead.  bytes: true when img8 holds the image (write it with
// rth_write_ppm_u8), false when img does.
int render_rccl(rth_scene *hs, const rt_camera &cam, int W, int H, int device, int gpus, HostImage &img,
                std::vector<unsigned char> &img8, bool want_floats, bool &bytes, std::vector<rt_stats> &st) {
    struct Dev {
        int id = 0;
        rt_scene *scene = nullptr;
        hipStream_t stream = nullptr;
        float *strip = nullptr, *recv = nullptr, *image = nullptr;
        unsigned char *strip8 = nullptr, *recv8 = nullptr, *image8 = nullptr;
        unsigned *flag = nullptr;
        int y0 = 0, step = 0, nrows = 0, rows_per = 0;
    };
    std::vector<Dev> d(gpus);
    std::vector<int> ids(gpus);
    std::vector<ncclComm_t> comms(gpus, nullptr);
    int rc = 0;
    auto fail = [&](const char *what, int code) {
        if (!rc) {
            std::cerr << "rt: " << what << " failed (" << code << ")" << std::endl;
            rc = 3;
        }
    };
    for (int g = 0; g < gpus && !rc; g++) {
        Dev &v = d[g];
        v.id = ids[g] = device + g;
        if (rth_row_set(H, gpus, g, kRowBlock, &v.y0, &v.step, &v.nrows, &v.rows_per)) fail("row set", -1);
        if (hipSetDevice(v.id) != hipSuccess) fail("hipSetDevice", v.id);
        int e = rt_scene_create(v.id, rth_desc(hs), &v.scene);
        if (!e) set_counters(v.scene, g_counters);
        if (e) fail(rt_strerror(e), e);
        const size_t strip = (size_t)v.rows_per * W * 3 * sizeof(float);
        const size_t strip8 = ((size_t)v.rows_per * W * 3 + 3) / 4 * 4;      // rt_quantize_u8: 4-B aligned
        if (!rc && (hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking) != hipSuccess ||
                    hipMalloc(&v.strip, strip) != hipSuccess || hipMalloc(&v.strip8, strip8) != hipSuccess ||
                    hipMalloc(&v.flag, sizeof(unsigned)) != hipSuccess ||
                    hipMemsetAsync(v.flag, 0, sizeof(unsigned), v.stream) != hipSuccess))
            fail("device buffers", g);
        if (!rc && g == 0 && (hipMalloc(&v.recv, strip * gpus) != hipSuccess ||
                              hipMalloc(&v.image, (size_t)W * H * 3 * sizeof(float)) != hipSuccess ||
                              hipMalloc(&v.recv8, strip8 * gpus) != hipSuccess ||
                              hipMalloc(&v.image8, (size_t)W * H * 3) != hipSuccess))
            fail("gather buffers", g);
    }
    if (!rc) {
        ncclResult_t r = ncclCommInitAll(comms.data(), gpus, ids.data());
        if (r != ncclSuccess) fail(ncclGetErrorString(r), (int)r);
    }
    for (int g = 0; g < gpus && !rc; g++) {
        Dev &v = d[g];
        (void)hipSetDevice(v.id);
        if (v.nrows > 0) {
            int e = rt_render_row_blocks_async(v.scene, &cam, W, H, v.y0, kRowBlock, v.step, v.nrows, v.strip,
                                               v.stream);
            if (e) fail(rt_strerror(e), e);
            // the writer's values as bytes, on the device, after the render
            if (!rc && !want_floats) {
                e = rt_quantize_u8(v.strip, (long long)v.nrows * W * 3, v.strip8, v.flag, v.stream);
                if (e) fail(rt_strerror(e), e);
            }
        }
    }
    // every device's flag (4 bytes each): the bytes are the writer's only when
    // no value anywhere is outside 0..255
    bytes = !want_floats;
    for (int g = 0; g < gpus && !rc && bytes; g++) {
        unsigned f = 0;
        (void)hipSetDevice(d[g].id);
        if (hipMemcpyAsync(&f, d[g].flag, sizeof f, hipMemcpyDeviceToHost, d[g].stream) != hipSuccess ||
            hipStreamSynchronize(d[g].stream) != hipSuccess)
            fail("flag copy", g);
        if (f & 1u) bytes = false;
    }
    if (!rc) {
        const size_t count = (size_t)d[0].rows_per * W * 3;
        ncclGroupStart();
        for (int g = 0; g < gpus; g++) {
            if (bytes)
                ncclGather(d[g].strip8, g == 0 ? d[0].recv8 : nullptr, count, ncclUint8, 0, comms[g], d[g].stream);
            else
                ncclGather(d[g].strip, g == 0 ? d[0].recv : nullptr, count, ncclFloat32, 0, comms[g], d[g].stream);
        }
        ncclResult_t r = ncclGroupEnd();
        if (r != ncclSuccess) fail(ncclGetErrorString(r), (int)r);
    }
    if (!rc && bytes) {
        (void)hipSetDevice(d[0].id);
        int e = rt_deinterleave_rows_u8(d[0].recv8, gpus, d[0].rows_per, W, H, kRowBlock, d[0].image8, d[0].stream);
        if (e) fail(rt_strerror(e), e);
        img8.resize((size_t)W * H * 3);
        if (!rc && (hipMemcpyAsync(img8.data(), d[0].image8, img8.size(), hipMemcpyDeviceToHost, d[0].stream) !=
                        hipSuccess ||
                    hipStreamSynchronize(d[0].stream) != hipSuccess))
            fail("image copy", 0);
    } else if (!rc) {
        (void)hipSetDevice(d[0].id);
        int e = rt_deinterleave_rows(d[0].recv, gpus, d[0].rows_per, W, H, kRowBlock, d[0].image, d[0].stream);
        if (e) fail(rt_strerror(e), e);
        if (!rc && (hipMemcpyAsync(img.data(), d[0].image, img.size() * sizeof(float), hipMemcpyDeviceToHost,
                                   d[0].stream) != hipSuccess ||
                    hipStreamSynchronize(d[0].stream) != hipSuccess))
            fail("image copy", 0);
    }
    for (int g = 0; g < gpus; g++) {
        Dev &v = d[g];
        (void)hipSetDevice(v.id);
        if (v.stream) (void)hipStreamSynchronize(v.stream);
        if (!rc && v.scene && v.nrows > 0 && rt_scene_last_stats(v.scene, &st[g])) fail("stats", g);
        if (comms[g]) ncclCommDestroy(comms[g]);
        if (v.strip) (void)hipFree(v.strip);
        if (v.recv) (void)hipFree(v.recv);
        if (v.image) (void)hipFree(v.image);
        if (v.strip8) (void)hipFree(v.strip8);
        if (v.recv8) (void)hipFree(v.recv8);
        if (v.image8) (void)hipFree(v.image8);
        if (v.flag) (void)hipFree(v.flag);
        if (v.stream) (void)hipStreamDestroy(v.stream);
        if (v.scene) rt_scene_destroy(v.scene);
    }
    return rc;
}

}  // namespace

int main(int argc, char *argv[]) {
    if (argc <= 1) {
        std::cout << "Error: Incorrect number of arguments in input file. Please follow this formate: imsize width height"
                  << std::endl;
        return 0;
    }
    const auto t_start = Clock::now();
    int depth = -1, W = -1, H = -1, gpus = 1, device = 0;
    bool stats = false;
    const char *stats_json = nullptr;
    std::string gather;
    const char *float_out = nullptr;
    for (int i = 2; i < argc; i++) {
        std::string a = argv[i];
        if (a == "--depth" && i + 1 < argc) depth = atoi(argv[++i]);
        else if (a == "--imsize" && i + 2 < argc) W = atoi(argv[++i]), H = atoi(argv[++i]);
        else if (a == "--gpus" && i + 1 < argc) gpus = atoi(argv[++i]);
        else if (a == "--device" && i + 1 < argc) device = atoi(argv[++i]);
        else if (a == "--float-out" && i + 1 < argc) float_out = argv[++i];
        else if (a == "--gather" && i + 1 < argc) gather = argv[++i];
        else if (a == "--stats") stats = true;
        else if (a == "--stats-json" && i + 1 < argc) stats_json = argv[++i];
    }
    // phases of the one-shot run (--stats-json), host clock
    double ph_parse = 0, ph_create = 0, ph_bvh = 0, ph_render = 0, ph_d2h = 0, ph_write = 0;
    // The HIP runtime and the device's context start on a thread of their
    // own while the scene file is parsed (C5's 11 MB: ~35 ms, HIP's start
    // 50-130 ms): neither needs the other
    int ndev = 0;
    double init_ms = 0.0;
    std::thread hip_init([&] {
        const auto ti = Clock::now();
        ndev = rt_device_count();                // the HIP runtime starts here
        // and the device's lazily made state (rt_device_init: context, memory,
        // copy paths, a hardware queue, the code object), for every device used
        for (int g = 0; g < std::max(1, gpus) && device + g < ndev; g++)
            if (device + g >= 0) (void)rt_device_init(device + g);
        init_ms = ms_since(ti);
    });
    auto t = Clock::now();
    rth_scene *hs = nullptr;
    std::vector<char> msg(1 << 16);
    int rc = rth_parse_file(argv[1], &hs, msg.data(), (int)msg.size());
    ph_parse = ms_since(t);
    if (rc != 0) hip_init.join();
    if (rc > 0) {
        std::cout << msg.data() << std::endl;
        return 0;
    }
    if (rc < 0) {
        std::string m(msg.data());
        size_t cut = m.rfind('\n');
        if (cut != std::string::npos) std::cerr << m.substr(0, cut) << std::endl;
        std::string what = cut == std::string::npos ? m : m.substr(cut + 1);
        if (rc == -2) throw std::out_of_range(what);
        throw std::invalid_argument(what);
    }
    if (depth >= 0) rth_set_depth(hs, depth);
    if (W > 1 && H > 1) rth_set_imsize(hs, W, H);
    W = rth_width(hs);
    H = rth_height(hs);
    rt_camera cam;
    rth_camera(hs, W, H, &cam);

    t = Clock::now();
    hip_init.join();
    const double ph_hip_init = ms_since(t);      // what the parse did not hide of init_ms
    if (ndev < 1) {
        std::cerr << "rt: no HIP device" << std::endl;
        return 2;
    }
    if (device < 0 || device >= ndev) {
        std::cerr << "rt: --device " << device << " out of range (" << ndev << " HIP device"
                  << (ndev == 1 ? "" : "s") << ")" << std::endl;
        return 2;
    }
    if (gpus < 1) gpus = 1;
    if (gpus > ndev - device) gpus = ndev - device;
    if (gather.empty()) gather = "host";
    if (gather != "rccl" && gather != "host") {
        std::cerr << "rt: --gather must be rccl or host" << std::endl;
        return 2;
    }
    t = Clock::now();
    g_counters = stats || stats_json;
    char out[4096];
    rth_output_path(argv[1], out, sizeof out);
    HostImage img((size_t)W * H * 3);
    double ph_count = 0.0;                 // the counting render (--stats*): not a phase of the run
    bool streamed = false;                 // one device: write_ppm_bytes or stream_ppm wrote the file
    int streamed_wr = 0;
    bool d2h_overlapped = false;           // the copy ran under the writer (its time is inside the write)
    const char *ppm_from = "floats";       // what the writer formatted: device-quantised bytes or floats
    const double ph_alloc = ms_since(t);
    std::vector<rt_stats> st(gpus);
    std::vector<int> rcs(gpus, 0);
    std::vector<std::thread> pool;
    std::vector<unsigned char> img8;      // --gather rccl: the writer's values as bytes, when they all fit
    bool rccl_bytes = false;
    if (gather == "rccl") {
        t = Clock::now();
        int r = render_rccl(hs, cam, W, H, device, gpus, img, img8, float_out || std::getenv("RT_PPM_FLOATS"),
                            rccl_bytes, st);
        if (r) return r;
        ph_render = ms_since(t);
        ppm_from = rccl_bytes ? "bytes" : "floats";
    }
    // --gather host: one host thread per device.  One device renders the image
    // in one call; several deal the rows out in 8-row blocks, round robin
    // (device g gets blocks g, g+N, ...: every device the same mix of cheap
    // and costly rows), each renders its row set into a buffer of its own and
    // the blocks are put back in image order on the host.
    // One device: each phase on its own, for --stats-json -- the scene upload,
    // the BVH (rt_scene_prepare), the render into HBM, one device->host copy.
    if (gather == "host" && gpus == 1) {
        rt_scene *s = nullptr;
        float *dimg = nullptr;
        t = Clock::now();
        int r = rt_scene_create(device, rth_desc(hs), &s);
        if (!r) set_counters(s, false);    // the timed render: no counters (they come from a second one)
        ph_create = ms_since(t);
        t = Clock::now();
        if (!r) r = rt_scene_prepare(s, &cam, W, H);
        ph_bvh = ms_since(t);
        if (!r && hipMalloc(&dimg, img.size() * sizeof(float)) != hipSuccess) r = RT_E_NOMEM;
        t = Clock::now();
        if (!r) r = rt_render_rows(s, &cam, W, H, 0, H, dimg, &st[0]);
        ph_render = ms_since(t);
        t = Clock::now();
        // below 512 MB of floats: the writer's values as bytes, quantised on
        // the device (3 B per pixel to the host); the floats when some value
        // is not 0..255, or --float-out wants them, or the image is large
        // enough for the pinned copy-and-write overlap below (C4, C5: it
        // hides the copy entirely)
        const bool big = (size_t)W * H * 3 * sizeof(float) >= (size_t(512) << 20);
        int bytes_rc = 1;
        if (!r && !float_out && !big && !std::getenv("RT_PPM_FLOATS")) {
            double d2h = 0.0;
            bytes_rc = write_ppm_bytes(out, dimg, W, H, r, d2h);
            if (bytes_rc != 1) {           // written (or failed): one phase, reported as the write
                streamed = true;
                streamed_wr = bytes_rc;
                ph_d2h = d2h;
                ph_write = ms_since(t) - d2h;
            }
        }
        t = Clock::now();
        // floats: copy and write overlapped (stream_ppm) for images of 512 MB
        // and more: below that the two pinned buffers' allocation costs more
        // than the overlap saves (C3's 201 MB: 37 -> 96 ms; C5's 3.2 GB: 542 ->
        // 361 ms)
        const bool stream = big || std::getenv("RT_PPM_BLOCK_ROWS") != nullptr;
        if (streamed || r) {
        } else if (!float_out && stream) {
            // one phase, reported as the write
            streamed = true;
            streamed_wr = stream_ppm(out, dimg, W, H, r);
            ph_write = ms_since(t);
            ph_d2h = 0.0;
            d2h_overlapped = true;
        } else {
            if (hipMemcpy(img.data(), dimg, img.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
                r = RT_E_HIP;
            ph_d2h = ms_since(t);
        }
        ppm_from = bytes_rc == 1 ? "floats" : "bytes";
        // --stats / --stats-json: the counts from one more render by the
        // counting instantiation, outside the phases (its image is the same)
        if (!r && g_counters) {
            const auto tc = Clock::now();
            rt_stats timed = st[0];
            set_counters(s, true);
            r = rt_render_rows(s, &cam, W, H, 0, H, dimg, &st[0]);
            st[0].kernel_ms = timed.kernel_ms;
            ph_count = ms_since(tc);
        }
        if (dimg) (void)hipFree(dimg);
        rt_scene_destroy(s);
        rcs[0] = r;
    }
    t = Clock::now();
    for (int g = 0; g < gpus && gather == "host" && gpus > 1; g++) {
        pool.emplace_back([&, g] {
            rt_scene *s = nullptr;
            int r = rt_scene_create(device + g, rth_desc(hs), &s);
            if (!r) set_counters(s, g_counters);
            if (!r) {
                std::vector<int> rows;
                for (int b = g * kRowBlock; b < H; b += gpus * kRowBlock)
                    for (int y = b; y < std::min(H, b + kRowBlock); y++) rows.push_back(y);
                if (!rows.empty()) {
                    std::vector<float> part(rows.size() * (size_t)W * 3);
                    r = rt_render_row_blocks(s, &cam, W, H, g * kRowBlock, kRowBlock, gpus * kRowBlock,
                                             (int)rows.size(), part.data(), &st[g]);
                    for (size_t k = 0; !r && k < rows.size(); k++)
                        std::copy(part.begin() + k * (size_t)W * 3, part.begin() + (k + 1) * (size_t)W * 3,
                                  img.begin() + (size_t)rows[k] * W * 3);
                }
            }
            rt_scene_destroy(s);
            rcs[g] = r;
        });
    }
    for (auto &th : pool) th.join();
    if (gpus > 1) ph_render = ms_since(t);      // scene, BVH, render and copies of every device
    for (int g = 0; g < gpus; g++) {
        if (rcs[g]) {
            std::cerr << "rt: render failed on device " << device + g << ": " << rt_strerror(rcs[g]) << std::endl;
            return 3;
        }
    }
    if (stats) {
        unsigned long long tot[4] = {0, 0, 0, 0};
        double ms = 0;
        for (auto &s : st) {
            tot[0] += s.primary, tot[1] += s.shadow, tot[2] += s.refraction, tot[3] += s.reflection;
            ms = std::max(ms, s.kernel_ms);
        }
        fprintf(stderr, "rays primary=%llu shadow=%llu refraction=%llu reflection=%llu kernel_ms=%.3f Mrays/s=%.1f\n",
                tot[0], tot[1], tot[2], tot[3], ms, (tot[0] + tot[1] + tot[2] + tot[3]) / (ms * 1e3));
    }
    if (float_out) {
        FILE *f = fopen(float_out, "wb");
        if (f) {
            fwrite(img.data(), sizeof(float), img.size(), f);
            fclose(f);
        }
    }
    int wr = streamed_wr;
    if (!streamed) {
        t = Clock::now();
        wr = rccl_bytes ? rth_write_ppm_u8(out, img8.data(), W, H, 0) : rth_write_ppm(out, img.data(), W, H, 0);
        ph_write = ms_since(t);
    }
    if (wr != 0) {
        std::cout << "ERROR: failed to create ppm image" << std::endl;
        return 0;
    }
    const int eff_depth = rth_desc(hs)->depth;
    rth_free(hs);
    if (stats_json) {
        unsigned long long tot[4] = {0, 0, 0, 0};
        double kms = 0, bvh_host = 0;
        for (auto &s : st) {
            tot[0] += s.primary, tot[1] += s.shadow, tot[2] += s.refraction, tot[3] += s.reflection;
            kms = std::max(kms, s.kernel_ms);
            bvh_host = std::max(bvh_host, s.bvh_build_ms);
        }
        long long ppm_bytes = 0;
        if (FILE *f = fopen(out, "rb")) {
            fseek(f, 0, SEEK_END);
            ppm_bytes = ftell(f);
            fclose(f);
        }
        const double total = ms_since(t_start) - ph_count;
        const unsigned long long rays = tot[0] + tot[1] + tot[2] + tot[3];
        FILE *f = std::strcmp(stats_json, "-") == 0 ? stderr : fopen(stats_json, "w");
        if (f) {
            fprintf(f,
                    "{\"scene\": \"%s\", \"imsize\": [%d, %d], \"depth\": %d, \"gpus\": %d, \"gather\": \"%s\", "
                    "\"rays\": %llu, \"hip_init_thread_ms\": %.3f, \"phases_ms\": {\"parse\": %.3f, \"hip_init\": %.3f, \"host_image_alloc\": %.3f, "
                    "\"scene_upload\": %.3f, \"bvh_build\": %.3f, "
                    "\"bvh_build_host\": %.3f, \"render\": %.3f, \"kernel\": %.3f, \"d2h\": %.3f, "
                    "\"quantise_ppm_write\": %.3f}, \"d2h_overlapped_with_write\": %s, \"ppm_from\": \"%s\", \"count_render_ms\": %.3f, "
                    "\"total_ms\": %.3f, \"ppm_bytes\": %lld, "
                    "\"Mrays_per_s_end_to_end\": %.3f, \"Mrays_per_s_kernel\": %.3f}\n",
                    argv[1], W, H, eff_depth, gpus, gather.c_str(), rays, init_ms, ph_parse, ph_hip_init, ph_alloc, ph_create, ph_bvh, bvh_host, ph_render,
                    kms, ph_d2h, ph_write, d2h_overlapped ? "true" : "false", ppm_from, ph_count, total, ppm_bytes, rays / (total * 1e3), kms > 0 ? rays / (kms * 1e3) : 0.0);
            if (f != stderr) fclose(f);
        }
    }
    return 0;
}
