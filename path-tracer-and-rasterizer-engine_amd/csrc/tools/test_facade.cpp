// test_facade — exercises the C++ path_tracer facade the way IoniqRE's application drives the
// reference engine (application.cu:66-99, renderer.cu:45-68): cadence, deferred reset, present.
// Prints one JSON line that tests/test_gpu_facade.py checks against the C-ABI path.
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "path_tracer.hpp"

#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

int main(int argc, char** argv) {
    const std::string ppm = argc > 1 ? argv[1] : "facade.ppm";
    try {
        // unknown presets surface as exceptions with the C-ABI status (ioniq_exception style)
        bool threw = false;
        try {
            iqpt::scene bad;
            bad.add_preset("no-such-preset");
        } catch (const iqpt::iqpt_exception& e) {
            threw = e.status() == IQPT_ERR_INVALID_ARG && std::string(e.what()).find("no-such-preset") != std::string::npos;
        }
        CHECK(threw);

        iqpt::camera cam(96, 64);
        iqpt::scene scn;
        scn.add_preset("cornell");
        iqpt::path_tracer_options opt;
        opt.max_depth = 8;
        opt.ppm_path = ppm;
        iqpt::path_tracer::init(&cam, opt);
        iqpt::path_tracer* pt = iqpt::path_tracer::get();
        CHECK(pt != nullptr);
        std::vector<iqpt::shader> shaders;
        // dt below the 0.1 s cadence: no launch (path_tracer.cu:378)
        pt->begin_frame();
        pt->draw_scene(scn, shaders, 0.05f);
        pt->end_frame();
        CHECK(pt->frames() == 0);
        CHECK(!scn.modified() == false);       // packet not built yet
        // 4 launches of 1 spp each
        for (int i = 0; i < 4; ++i) {
            pt->begin_frame();
            pt->draw_scene(scn, shaders, 0.2f);
            pt->end_frame();
        }
        CHECK(pt->frames() == 4);
        CHECK(!scn.modified());
        std::vector<float> lin4;
        pt->read_linear(lin4);
        // deferred reset: the next launch restarts the mean at frame 1
        pt->reset();
        pt->begin_frame();
        pt->draw_scene(scn, shaders, 0.2f);
        pt->end_frame();
        CHECK(pt->frames() == 1);
        std::vector<float> lin5;
        pt->read_linear(lin5);
        double s4 = 0.0, s5 = 0.0;
        for (size_t i = 0; i < lin4.size(); i += 4) {
            s4 += (double)lin4[i] + lin4[i + 1] + lin4[i + 2];
            s5 += (double)lin5[i] + lin5[i + 1] + lin5[i + 2];
        }
        // one more cadence tick makes end_frame present the launched frame as PPM
        pt->begin_frame();
        pt->draw_scene(scn, shaders, 0.2f);
        pt->end_frame();
        FILE* f = std::fopen(ppm.c_str(), "rb");
        CHECK(f != nullptr);
        std::fclose(f);
        std::printf("{\"ok\": true, \"sum_after_4\": %.9g, \"sum_after_reset\": %.9g, \"rays\": %llu}\n", s4, s5,
                    (unsigned long long)pt->rays_traced());
        iqpt::path_tracer::shutdown();
        CHECK(iqpt::path_tracer::get() == nullptr);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
