// asw_stereo — command-line host driver: the reference main.cpp's ASW flow on the
// MI355X library, through the C-ABI of include/asw.h only.
//
// Mirrors stereo_matching/main.cpp:
//   * pics.txt lists image paths, two per pair (left, right) (main.cpp:136-147);
//     the output folder of a pair is its left path up to the first '/'
//     (main.cpp:150-155);
//   * images are decoded to RGBA8 (lodepng::decode in the reference,
//     main.cpp:183-186; png_io.cpp here);
//   * every pair runs `runs` times (main.cpp:213: 10) and the per-stage times of
//     each run go to a TSV file named after the device (main.cpp:164-166, 181,
//     634-708), here from HIP events (asw_timings);
//   * outputs: <folder>/asw_consistency_pre-reff.png (the reference's file of the
//     same name, main.cpp:625-627), asw_consistency.png (its `consistency_error`
//     image before refinement), asw_wta_disparity.png (its `asw_left_wta` image)
//     and, with the k = 6 refinement iterations of main.cpp:540-617 (--refine K,
//     0 = off), asw_disparity.png (refined + 3x3 median, main.cpp:619-623) and
//     asw_consistency_post-reff.png (main.cpp:629-631);
//   * errors are printed and the driver continues with the next pair, like ErCheck
//     (main.cpp:27-30);
//   * beyond the reference: --devices I,J,... splits the disparity range of every
//     pair across several GPUs (asw_create_multi: RCCL all-reduces for the WTA; a
//     repeated id puts several shards on one GPU), and 16-bit disparity images
//     (asw_wta_disparity16.png, asw_consistency16.png with 65535 = inconsistent) are
//     written with --png16 and always when D > 256, where the 8-bit codes collide
//     (the LR check then compares indices, ASW_LR_NATIVE).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "asw.h"
#include "png_io.h"

using asw_host::Image;

namespace {

struct Options {
    std::string pics = "pics.txt";
    std::string root;  // default: directory of pics
    std::string tsv;   // default: "<device name>.tsv" in the current directory
    int runs = 10, ndisp = 61, taps = 33, iters = 7, device = 0, refine = 6;
    std::vector<int> devices;  // --devices: one context over several GPUs
    float gamma_c = -1.0f, gamma_g = -1.0f, tau = -1.0f;
    bool lab = false, lr = true, native_lr = false, png16 = false;
};

void usage() {
    std::fprintf(stderr,
                 "usage: asw_stereo [--pics FILE] [--root DIR] [--runs N] [--ndisp D] [--taps T] [--iters R]\n"
                 "                  [--gamma-c G] [--gamma-g G] [--tau TAU] [--lab] [--no-lr] [--native-lr]\n"
                 "                  [--refine K] [--device I | --devices I,J,...] [--png16] [--tsv FILE]\n");
}

bool parse(int argc, char **argv, Options &o) {
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&](const char *what) -> const char * {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "%s needs a value\n", what);
                return nullptr;
            }
            return argv[++i];
        };
        const char *v = nullptr;
        if (a == "--pics") { if (!(v = next("--pics"))) return false; o.pics = v; }
        else if (a == "--root") { if (!(v = next("--root"))) return false; o.root = v; }
        else if (a == "--refine") { if (!(v = next("--refine"))) return false; o.refine = std::atoi(v); }
        else if (a == "--tsv") { if (!(v = next("--tsv"))) return false; o.tsv = v; }
        else if (a == "--runs") { if (!(v = next("--runs"))) return false; o.runs = std::atoi(v); }
        else if (a == "--ndisp") { if (!(v = next("--ndisp"))) return false; o.ndisp = std::atoi(v); }
        else if (a == "--taps") { if (!(v = next("--taps"))) return false; o.taps = std::atoi(v); }
        else if (a == "--iters") { if (!(v = next("--iters"))) return false; o.iters = std::atoi(v); }
        else if (a == "--device") { if (!(v = next("--device"))) return false; o.device = std::atoi(v); }
        else if (a == "--gamma-c") { if (!(v = next("--gamma-c"))) return false; o.gamma_c = (float)std::atof(v); }
        else if (a == "--gamma-g") { if (!(v = next("--gamma-g"))) return false; o.gamma_g = (float)std::atof(v); }
        else if (a == "--tau") { if (!(v = next("--tau"))) return false; o.tau = (float)std::atof(v); }
        else if (a == "--devices") {
            if (!(v = next("--devices"))) return false;
            o.devices.clear();
            for (const char *q = v; *q;) {
                char *end = nullptr;
                const long d = std::strtol(q, &end, 10);
                if (end == q) return false;
                o.devices.push_back((int)d);
                q = *end == ',' ? end + 1 : end;
            }
        }
        else if (a == "--png16") o.png16 = true;
        else if (a == "--lab") o.lab = true;
        else if (a == "--no-lr") o.lr = false;
        else if (a == "--native-lr") o.native_lr = true;
        else if (a == "-h" || a == "--help") { usage(); std::exit(0); }
        else { std::fprintf(stderr, "unknown argument %s\n", a.c_str()); return false; }
    }
    if (o.runs < 1) o.runs = 1;
    return true;
}

std::string dir_of(const std::string &path) {
    const size_t k = path.find_last_of('/');
    return k == std::string::npos ? std::string(".") : path.substr(0, k);
}

std::string join(const std::string &a, const std::string &b) {
    if (b.empty() || b[0] == '/') return b;
    return a.empty() || a == "." ? b : a + "/" + b;
}

bool read_pairs(const std::string &path, std::vector<std::string> &left, std::vector<std::string> &right) {
    FILE *fp = std::fopen(path.c_str(), "r");
    if (!fp) return false;
    std::vector<std::string> items;
    char buf[4096];
    while (std::fscanf(fp, "%4095s", buf) == 1) items.emplace_back(buf);
    std::fclose(fp);
    for (size_t i = 0; i + 1 < items.size(); i += 2) {
        left.push_back(items[i]);
        right.push_back(items[i + 1]);
    }
    return true;
}

}  // namespace

int main(int argc, char **argv) {
    Options o;
    if (!parse(argc, argv, o)) {
        usage();
        return 2;
    }
    if (asw_abi_version() != ASW_ABI_VERSION) {  // asw_outputs / asw_timings layouts (include/asw.h)
        std::fprintf(stderr, "libasw_hip.so has ABI revision %d, asw_stereo was built for %d: rebuild\n",
                     asw_abi_version(), ASW_ABI_VERSION);
        return 1;
    }
    if (o.root.empty()) o.root = dir_of(o.pics);
    std::vector<std::string> lefts, rights;
    if (!read_pairs(o.pics, lefts, rights)) {
        std::fprintf(stderr, "cannot read %s\n", o.pics.c_str());
        return 1;
    }
    if (o.devices.empty()) o.devices.push_back(o.device);
    char devname[256] = "hip-device";
    asw_device_name(o.devices[0], devname, (int)sizeof devname);
    if (o.devices.size() > 1) {
        const size_t k = std::strlen(devname);
        std::snprintf(devname + k, sizeof devname - k, " x%zu", o.devices.size());
    }
    std::printf("\t- Device name: %s\n", devname);
    const std::string tsv_path = o.tsv.empty() ? std::string(devname) + ".tsv" : o.tsv;
    FILE *tsv = std::fopen(tsv_path.c_str(), "w");
    if (!tsv) std::fprintf(stderr, "cannot write %s (timings go to stdout only)\n", tsv_path.c_str());

    int failures = 0;
    for (size_t k = 0; k < lefts.size(); ++k) {
        const std::string folder = lefts[k].substr(0, lefts[k].find('/'));
        std::printf("\n%s\n", folder.c_str());
        Image L, R;
        std::string e = asw_host::png_load(join(o.root, lefts[k]), L);
        if (e.empty()) e = asw_host::png_load(join(o.root, rights[k]), R);
        if (e.empty() && (L.width != R.width || L.height != R.height)) e = "left and right sizes differ";
        if (!e.empty()) {
            std::fprintf(stderr, "%s: %s\n", folder.c_str(), e.c_str());
            ++failures;
            continue;
        }
        asw_params p;
        asw_params_default(&p);
        p.width = (int)L.width;
        p.height = (int)L.height;
        p.ndisp = o.ndisp;
        p.taps = o.taps;
        p.iters = o.iters;
        if (o.gamma_c > 0) p.gamma_c = o.gamma_c;
        if (o.gamma_g > 0) p.gamma_g = o.gamma_g;
        if (o.tau > 0) p.tad_tau = o.tau;
        p.color_space = o.lab ? ASW_COLOR_LAB : ASW_COLOR_RGB;
        p.lr_check = o.lr ? 1 : 0;
        const bool wide = p.ndisp > 256;  // 8-bit codes collide: compare indices, write 16-bit images
        p.lr_mode = (o.native_lr || wide) ? ASW_LR_NATIVE : ASW_LR_U8;
        const bool png16 = o.png16 || wide;
        asw_ctx *ctx = nullptr;
        int st = o.devices.size() > 1 ? asw_create_multi(&p, o.devices.data(), (int)o.devices.size(), &ctx)
                                      : asw_create(&p, o.devices[0], &ctx);
        if (st != ASW_OK) {
            std::fprintf(stderr, "%s: asw_create: %s (hip %d)\n", folder.c_str(), asw_strerror(st),
                         asw_last_hip_error());
            ++failures;
            continue;
        }
        // the loop runs on d-sharded contexts too (asw_set_refine: its asw_WTA_REF scan is
        // exchanged like the WTA); it feeds back 8-bit codes, so D > 256 has none
        const bool refine = o.refine > 0 && p.lr_check && !wide;
        if (o.refine > 0 && !refine)
            std::fprintf(stderr, "%s: refinement skipped (%s)\n", folder.c_str(),
                         !p.lr_check ? "it needs the LR check" : "D > 256: the loop re-reads 8-bit codes");
        if (refine) {
            asw_refine_params rp;
            asw_refine_params_default(&rp);
            rp.iters = o.refine;
            st = asw_set_refine(ctx, &rp);
            if (st != ASW_OK) {
                std::fprintf(stderr, "%s: asw_set_refine: %s\n", folder.c_str(), asw_strerror(st));
                ++failures;
                asw_destroy(ctx);
                continue;
            }
        }
        const size_t S = (size_t)p.width * p.height;
        std::vector<uint8_t> disp(S * 4), lr(S * 4), lr_red(S * 4), fin(S * 4), post(S * 4);
        std::vector<uint16_t> disp16(png16 ? S : 0), lr16(png16 ? S : 0);
        asw_outputs out;
        std::memset(&out, 0, sizeof out);
        out.disp_rgba = disp.data();
        out.lr_rgba = lr.data();
        out.lr_red_rgba = lr_red.data();
        out.final_rgba = refine ? fin.data() : nullptr;
        out.post_red_rgba = refine ? post.data() : nullptr;
        out.disp16 = png16 ? disp16.data() : nullptr;
        out.lr16 = png16 && p.lr_check ? lr16.data() : nullptr;
        if (tsv) {
            std::fprintf(tsv, "\n%s - %s\n", devname, folder.c_str());
            std::fprintf(tsv, "id\taggr\tsupp_w\tv_aggr_mean\th_aggr_mean\ttotal aggregation\twta\tconsistency\t"
                              "total\trefine\th2d\td2h\texchange\n");
        }
        for (int run = 0; run < o.runs && st == ASW_OK; ++run) {
            asw_timings t;
            std::memset(&t, 0, sizeof t);
            st = asw_match(ctx, L.rgba.data(), R.rgba.data(), &out, &t);
            if (st != ASW_OK) break;
            std::printf("run %d: total %.3f ms (aggregation %.3f, V %.3f, H %.3f per pass)\n", run, t.total,
                        t.aggregation_total, t.v_pass_mean, t.h_pass_mean);
            if (tsv)
                std::fprintf(tsv, "%d\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\t%0.3f\n",
                             run, t.raw_cost, t.support, t.v_pass_mean, t.h_pass_mean, t.aggregation_total, t.wta,
                             t.consistency, t.total, t.refine, t.h2d, t.d2h, t.exchange);
        }
        asw_destroy(ctx);
        if (st != ASW_OK) {
            std::fprintf(stderr, "%s: asw_match: %s (hip %d)\n", folder.c_str(), asw_strerror(st),
                         asw_last_hip_error());
            ++failures;
            continue;
        }
        const std::string dir = join(o.root, folder);
        struct {
            const char *name;
            const std::vector<uint8_t> *img;
        } outs[] = {{"asw_wta_disparity.png", &disp},
                    {"asw_consistency.png", &lr},
                    {"asw_consistency_pre-reff.png", &lr_red},
                    {"asw_disparity.png", &fin},
                    {"asw_consistency_post-reff.png", &post}};
        for (const auto &w : outs) {
            if (!p.lr_check && w.img != &disp) continue;
            if (!refine && (w.img == &fin || w.img == &post)) continue;
            e = asw_host::png_save(dir + "/" + w.name, w.img->data(), L.width, L.height, 4);
            if (!e.empty()) {
                std::fprintf(stderr, "%s: %s\n", folder.c_str(), e.c_str());
                ++failures;
            }
        }
        if (png16) {
            e = asw_host::png_save16(dir + "/asw_wta_disparity16.png", disp16.data(), L.width, L.height);
            if (e.empty() && p.lr_check)
                e = asw_host::png_save16(dir + "/asw_consistency16.png", lr16.data(), L.width, L.height);
            if (!e.empty()) {
                std::fprintf(stderr, "%s: %s\n", folder.c_str(), e.c_str());
                ++failures;
            }
        }
    }
    if (tsv) std::fclose(tsv);
    return failures ? 1 : 0;
}
