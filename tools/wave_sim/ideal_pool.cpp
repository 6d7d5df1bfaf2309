// Upper bound of a ray pool: lanes never wait for shading -- a finished
// ray goes to a shade queue and the lane takes a ready ray at once; shade passes run 64
// rays -- with no cost for moving rays.  Node / leaf pass policy as the kernel's.
// g++ -O2 -o ideal_pool ideal_pool.cpp && ./ideal_pool trace [leaf_batch] [node_steps]
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <deque>
#include <algorithm>
using namespace std;
struct Trace { vector<uint8_t> tok; vector<uint32_t> ray_start; vector<uint32_t> path_start; };
static Trace load(const char* f) {
    FILE* fp = fopen(f, "rb"); fseek(fp, 0, SEEK_END); long n = ftell(fp); fseek(fp, 0, SEEK_SET);
    vector<char> b(n); if (fread(b.data(), 1, n, fp) != (size_t)n) exit(1); fclose(fp);
    Trace t; t.tok.reserve(n);
    for (long i = 0; i < n; i++) {
        char c = b[i];
        if (c == 'P') t.path_start.push_back(t.ray_start.size());
        else if (c == 'R') t.ray_start.push_back(t.tok.size());
        else if (c == 'N') t.tok.push_back(0);
        else if (c == 'U' || c == 'W') i++;  // (a rejection loop's candidate count: not used here)
        else if (c == 'a' || c == 'o' || c == 'g' || c == 'h') {  // a sphere test (a leaf run of two: one token)
            const char d = i + 1 < n ? b[i + 1] : 0;
            if (d == 'a' || d == 'o' || d == 'g' || d == 'h') { t.tok.push_back(2); i++; } else t.tok.push_back(1);
        }
    }
    t.ray_start.push_back(t.tok.size()); t.path_start.push_back(t.ray_start.size() - 1);
    return t;
}
int main(int argc, char** argv) {
    Trace t = load(argv[1]);
    int leaf_batch = argc > 2 ? atoi(argv[2]) : 12, steps = argc > 3 ? atoi(argv[3]) : 8;
    const uint32_t npaths = t.path_start.size() - 1;
    // path work list: (path, ray) pairs ready to trace
    struct R { uint32_t path, ray; };
    deque<R> ready; uint32_t next_path = 0;
    auto fill = [&]() { while (ready.size() < 256 && next_path < npaths) ready.push_back({next_path++, 0}); };
    fill();
    bool busy[64] = {}; R cur[64]; uint32_t pos[64], end[64];
    double wsteps = 0, slanes = 0, lpasses = 0, llanes = 0, npasses = 0, rays = 0, shade = 0, shq = 0;
    auto take = [&](int l) {
        if (ready.empty()) { busy[l] = false; return; }
        cur[l] = ready.front(); ready.pop_front(); uint32_t r = t.path_start[cur[l].path] + cur[l].ray;
        pos[l] = t.ray_start[r]; end[l] = t.ray_start[r + 1]; busy[l] = true; rays++;
    };
    for (int l = 0; l < 64; l++) take(l);
    vector<R> done;
    for (;;) {
        // finished lanes: to the shade queue, then a ready ray
        for (int l = 0; l < 64; l++) if (busy[l] && pos[l] >= end[l]) { done.push_back(cur[l]); take(l); }
        for (int l = 0; l < 64; l++) if (!busy[l]) take(l);
        while (done.size() >= 64 || (ready.empty() && next_path >= npaths && !done.empty())) {
            size_t k = min<size_t>(64, done.size()); shade++; shq += k;
            for (size_t i = 0; i < k; i++) {
                R x = done[i]; uint32_t nr = t.path_start[x.path + 1] - t.path_start[x.path];
                if (x.ray + 1 < nr) ready.push_back({x.path, x.ray + 1});
            }
            done.erase(done.begin(), done.begin() + k);
            fill();
            for (int l = 0; l < 64; l++) if (!busy[l]) take(l);
        }
        int ntr = 0, nlm = 0;
        for (int l = 0; l < 64; l++) if (busy[l] && pos[l] < end[l]) { ntr++; if (t.tok[pos[l]]) nlm++; }
        if (ntr == 0) { if (ready.empty() && next_path >= npaths && done.empty()) break; continue; }
        if (nlm == ntr || nlm >= leaf_batch) {
            lpasses++; llanes += nlm;
            for (int l = 0; l < 64; l++) if (busy[l] && pos[l] < end[l] && t.tok[pos[l]]) pos[l]++;
        } else {
            npasses++;
            for (int s = 0; s < steps; s++) {
                int a = 0;
                for (int l = 0; l < 64; l++) if (busy[l] && pos[l] < end[l] && !t.tok[pos[l]]) { a++; pos[l]++; }
                if (a) { wsteps++; slanes += a; }
            }
        }
    }
    printf("ideal pool leaf_batch %d: per ray wsteps %.4f (%.1f lanes) leaf passes %.4f (%.1f lanes) shade %.4f (%.1f)\n", leaf_batch,
           wsteps / rays, slanes / wsteps, lpasses / rays, llanes / lpasses, shade / rays, shq / shade);
    const double CN = getenv("CN") ? atof(getenv("CN")) : 60, CL = getenv("CL") ? atof(getenv("CL")) : 400,
                 CS = getenv("CS") ? atof(getenv("CS")) : 3500, CA = getenv("CA") ? atof(getenv("CA")) : 3000;
    // (camera rays: one get_ray pass per 64 ended paths -- the pool batches them too)
    const double paths = (double)npaths, cyc = wsteps * CN + lpasses * CL + shade * CS + paths / 64.0 * CA + npasses * 30;
    printf("model cycles/ray %.1f (node %.1f leaf %.1f shade %.1f cam %.1f)\n", cyc / rays, wsteps * CN / rays, lpasses * CL / rays,
           shade * CS / rays, paths / 64.0 * CA / rays);
}
