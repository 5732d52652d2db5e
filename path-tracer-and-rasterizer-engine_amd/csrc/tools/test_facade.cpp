// test_facade — exercises the C++ path_tracer facade the way IoniqRE's application drives the
// reference engine (application.cu:66-99, renderer.cu:45-68): cadence, deferred reset, present.
// Prints one JSON line that tests/test_gpu_facade.py checks against the C-ABI path.
#include <cmath>
#include <cstring>
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
        const unsigned long long rays = (unsigned long long)pt->rays_traced();
        iqpt::path_tracer::shutdown();
        CHECK(iqpt::path_tracer::get() == nullptr);

        // the sharded present path (one process per GPU; here a one-rank communicator): the frame comes back
        // through the RCCL gather and rank 0's assembly, and must equal the single-GPU facade's bit for bit
        auto run4 = [&](const iqpt::path_tracer_options& o, std::vector<float>& lin, std::vector<iqpt::path_tracer::pixel>& px) {
            iqpt::scene s;
            s.add_preset("cornell");
            iqpt::path_tracer::init(&cam, o);
            iqpt::path_tracer* p = iqpt::path_tracer::get();
            for (int i = 0; i < 5; ++i) {            // 4 launches; the 5th tick fetches the 4th launch's frame
                p->begin_frame();
                p->draw_scene(s, shaders, 0.2f);
                p->end_frame();
            }
            p->read_linear(lin);
            px = p->host_pixels();
            iqpt::path_tracer::shutdown();
        };
        iqpt::path_tracer_options single = opt;
        single.ppm_path.clear();
        iqpt::path_tracer_options sharded = single;
        sharded.rank = 0;
        sharded.world = 1;
        sharded.comm_id = iqpt::path_tracer::comm_unique_id();
        std::vector<float> lin_a, lin_b;
        std::vector<iqpt::path_tracer::pixel> px_a, px_b;
        run4(single, lin_a, px_a);
        run4(sharded, lin_b, px_b);
        CHECK(lin_a.size() == lin_b.size() && px_a.size() == px_b.size());
        CHECK(std::memcmp(lin_a.data(), lin_b.data(), lin_a.size() * sizeof(float)) == 0);
        CHECK(std::memcmp(px_a.data(), px_b.data(), px_a.size() * sizeof(px_a[0])) == 0);
        std::printf("{\"ok\": true, \"sum_after_4\": %.9g, \"sum_after_reset\": %.9g, \"rays\": %llu, \"sharded_equal\": true}\n",
                    s4, s5, rays);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
