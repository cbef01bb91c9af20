// tbdk_tbd_app — command-line front end of tbdk_app_run with the flags of the
// reference sample example_gpu_tbd (samples/gpu/tbd.cpp:145-331).
//
// The tracking flags behave as in the sample.  The image-path flags (HOG
// parameters, gray/resize, video output, the frame source) are accepted and
// ignored: with bbox files the tracker never reads pixels, and the frame loop
// runs --num_tracking_frames frames.  Without a bbox file the sample would run
// its HOG detector, which this tool does not provide (exit 1).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/tbdk.h"

static const char* kIgnored[] = {"--make_gray", "--resize_src", "--width", "--height", "--hit_threshold",
                                 "--scale", "--nlevels", "--win_width", "--win_stride_width",
                                 "--win_stride_height", "--block_width", "--block_stride_width",
                                 "--block_stride_height", "--cell_width", "--nbins", "--gr_threshold",
                                 "--gamma_correct", "--write_video", "--dst_video", "--dst_video_fps", "--video",
                                 "--camera", "--folder", "--svm"};

int main(int argc, char** argv)
{
    tbdk_app_args a;
    tbdk_app_default_args(&a);
    a.verbose = 1;
    std::string src;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) {
                std::printf("error: missing value for %s\n", k.c_str());
                std::exit(1);
            }
            return argv[++i];
        };
        bool ignored = false;
        for (const char* g : kIgnored)
            if (k == g) {
                next();
                ignored = true;
            }
        if (ignored) continue;
        if (k == "--help") {
            std::printf("tbdk_tbd_app: the tracking loop of example_gpu_tbd over bbox files\n"
                        "  --pedestrian_bbox_filename <f> --vehicle_bbox_filename <f>\n"
                        "  --write_tracking <true/false> --pedestrian_tracking_filepath <f>\n"
                        "  --vehicle_tracking_filepath <f> --history_distribution <a,b,...>\n"
                        "  --num_tracking_iters <int> --num_tracking_frames <int> [--seed <uint>]\n");
            return -1;
        } else if (k == "--history_distribution") {
            a.history_distribution = next();
        } else if (k == "--pedestrian_bbox_filename") {
            a.pedestrian_bbox_filename = next();
        } else if (k == "--vehicle_bbox_filename") {
            a.vehicle_bbox_filename = next();
        } else if (k == "--write_tracking") {
            a.write_tracking = std::string(next()) == "true";
        } else if (k == "--pedestrian_tracking_filepath") {
            a.pedestrian_tracking_filepath = next();
        } else if (k == "--vehicle_tracking_filepath") {
            a.vehicle_tracking_filepath = next();
        } else if (k == "--num_tracking_iters") {
            a.num_tracking_iters = std::atoi(next());
        } else if (k == "--num_tracking_frames") {
            a.num_tracking_frames = std::atoi(next());
        } else if (k == "--seed") {  // not in the sample: srand() before the run
            a.rand_seed = (uint32_t)std::strtoul(next(), nullptr, 10);
        } else if (src.empty()) {
            src = k;
        } else {
            std::printf("error: unknown key: %s\n", k.c_str());
            return 1;
        }
    }
    if (!a.pedestrian_bbox_filename && !a.vehicle_bbox_filename) {
        std::printf("error: no bbox file (the HOG detection path is not part of libtbdk)\n");
        return 1;
    }
    tbdk_app_result r;
    const int rc = tbdk_app_run(&a, &r);
    if (rc != TBDK_OK) {
        std::printf("error: tbdk_app_run failed (%d)\n", rc);
        return 1;
    }
    const char* names[2] = {"pedestrians", "vehicles"};
    for (int c = 0; c < 2; ++c) {
        if (!(c == 0 ? a.pedestrian_bbox_filename : a.vehicle_bbox_filename)) continue;
        const tbdk_scenario_metrics& m = r.scenario[c];
        std::printf("%s: frames %d MT %d PT %d ML %d IDSW %d FM %d MOTA %g A-MOTA %g MOTP %g\n", names[c], m.frames,
                    m.mt, m.pt, m.ml, m.idsw, m.fm, m.mota, m.amota, m.motp);
    }
    return 0;
}
