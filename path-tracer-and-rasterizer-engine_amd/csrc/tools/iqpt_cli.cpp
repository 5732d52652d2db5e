// iqpt_cli — headless stand-in for IoniqRE's application loop (application.cu:66-99) over the
// path_tracer facade: builds a preset scene, runs begin_frame / draw_scene / end_frame with a
// fixed dt, and dumps the frame as PPM (the D3D11 present path, path_tracer.cu:171-210, is out of
// scope). Usage:
//   iqpt_cli --preset cornell --width 1920 --height 1080 --spp 64 --max-depth 8 --out cornell.ppm
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "path_tracer.hpp"

int main(int argc, char** argv) {
    std::string preset = "cornell", out = "iqpt.ppm";
    int width = 640, height = 360, spp = 16, launches = 1, max_depth = 8, device = 0;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        const char* v = argv[i + 1];
        if (k == "--preset") preset = v;
        else if (k == "--out") out = v;
        else if (k == "--width") width = std::atoi(v);
        else if (k == "--height") height = std::atoi(v);
        else if (k == "--spp") spp = std::atoi(v);
        else if (k == "--launches") launches = std::atoi(v);
        else if (k == "--max-depth") max_depth = std::atoi(v);
        else if (k == "--device") device = std::atoi(v);
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 2;
        }
    }
    try {
        iqpt::camera cam((uint16_t)width, (uint16_t)height);
        iqpt::scene scn;
        scn.add_preset(preset);
        iqpt::path_tracer_options opt;
        opt.device = device;
        opt.max_depth = max_depth;
        opt.spp_per_launch = (uint32_t)spp;
        opt.launch_interval = 0.0f;
        opt.ppm_path = out;
        iqpt::path_tracer::init(&cam, opt);
        iqpt::path_tracer* pt = iqpt::path_tracer::get();
        std::vector<iqpt::shader> shaders;
        // each frame: the launch of frame k is read back at frame k+1 (path_tracer.cu:382-386)
        for (int f = 0; f <= launches; ++f) {
            pt->begin_frame();
            if (f < launches) {
                pt->draw_scene(scn, shaders, 1.0f);
            } else {
                std::vector<float> lin;
                pt->read_linear(lin);   // sync
                pt->draw_scene(scn, shaders, 0.0f);
            }
            pt->end_frame();
        }
        // final readback + dump of the last launch
        iqpt::path_tracer_options o2 = opt;
        (void)o2;
        std::vector<uint8_t> bgra((size_t)width * height * 4);
        IQPT_THROW_FAILED(iqpt_read(pt->context(), nullptr, bgra.data()));
        IQPT_THROW_FAILED(iqpt_write_ppm(out.c_str(), (uint32_t)width, (uint32_t)height, bgra.data()));
        std::printf("{\"preset\": \"%s\", \"frames\": %llu, \"rays\": %llu, \"out\": \"%s\"}\n", preset.c_str(),
                    (unsigned long long)pt->frames(), (unsigned long long)pt->rays_traced(), out.c_str());
        iqpt::path_tracer::shutdown();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
