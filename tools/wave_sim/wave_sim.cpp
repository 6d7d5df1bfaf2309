// Trace-driven model of the megakernel's wave scheduler (render.hip's loop), one wave at a
// time, on traces of the reference's traversal (trace_oracle.py): node passes of `steps`
// unrolled steps, leaf passes at `leaf_batch` lanes (two-sphere leaf runs as one token),
// shading at `shade_batch` finished lanes, chunk items of 16 samples.  Reports lanes per
// pass kind (calibrated against the stamps build: C4 node steps 40.7 vs 39.7 measured, leaf
// passes 36.5 vs 33.4, shade 57.3 vs 56.6), how often the leaf pass's root blocks run
// (the round-5 root rounds), the rejection loops' wave iterations, and a cost model
// (cycles per wave pass: CN, CL, CS, CA env vars; the defaults are rough).
// g++ -O2 -o wave_sim wave_sim.cpp && ./wave_sim trace [shade_batch leaf_batch steps cam_batch exit_k]
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>
#include <algorithm>
using namespace std;
// tokens: 0 = node, 1 = one sphere leaf, 2 = two sphere leaves (a leaf run)
struct Trace { vector<uint8_t> tok; vector<uint32_t> ray_start; vector<uint32_t> path_start; vector<uint8_t> uit, wit; };
static Trace load(const char* f) {
    FILE* fp = fopen(f, "rb"); fseek(fp, 0, SEEK_END); long n = ftell(fp); fseek(fp, 0, SEEK_SET);
    vector<char> b(n); fread(b.data(), 1, n, fp); fclose(fp);
    Trace t; t.tok.reserve(n);
    for (long i = 0; i < n; i++) {
        char c = b[i];
        if (c == 'P') { t.path_start.push_back(t.ray_start.size()); t.wit.push_back(0); }
        else if (c == 'R') { t.ray_start.push_back(t.tok.size()); t.uit.push_back(0); }
        else if (c == 'U') { t.uit.back() = (uint8_t)b[++i]; }
        else if (c == 'W') { t.wit.back() = (uint8_t)b[++i]; }
        else if (c == 'N') t.tok.push_back(0);
        else if (c == 'a' || c == 'o' || c == 'g' || c == 'h') {
            auto oc = [](char x) { return x == 'a' ? 0 : x == 'o' ? 1 : x == 'g' ? 2 : 3; };
            char d = i + 1 < n ? b[i + 1] : 0;
            if (d == 'a' || d == 'o' || d == 'g' || d == 'h') { t.tok.push_back(32 + oc(c) * 4 + oc(d)); i++; }
            else t.tok.push_back(16 + oc(c));
        }
    }
    t.ray_start.push_back(t.tok.size());
    t.path_start.push_back(t.ray_start.size() - 1);
    return t;
}
struct Stats { double iters=0, node_passes=0, node_pass_lanes=0, wsteps=0, step_lanes=0, leaf_passes=0, leaf_lanes=0,
    shade_passes=0, shade_lanes=0, early=0, w_max=0, w_sum=0, w_coop=0, u_passes=0, u_lanes=0, u_max=0, u_sum=0, b_sq1=0, b_sq2=0, b_dv1=0, b_dv2=0, b_both=0, b_any=0, b_2nd=0, adv=0, adv_lanes=0, rays=0, spheres=0, nodes=0; };
enum { NEED, CAM, TRACE, SHADE, DONE };
static double coop_rounds(const Trace&, uint32_t*, int*, int, int) { return 0; }
struct P { int shade_batch=52, leaf_batch=12, steps=8, chunk=16, spp=512, claim=32, adv_min=1, exit_k=0; };
int main(int argc, char** argv) {
    Trace t = load(argv[1]);
    P p; if (argc > 2) p.shade_batch = atoi(argv[2]); if (argc > 3) p.leaf_batch = atoi(argv[3]); if (argc > 4) p.steps = atoi(argv[4]); if (argc > 5) p.adv_min = atoi(argv[5]); if (argc > 6) p.exit_k = atoi(argv[6]);
    const uint32_t npaths = t.path_start.size() - 1, npix = npaths / p.spp, cpp = p.spp / p.chunk;
    const uint32_t nitems = npix * cpp;
    fprintf(stderr, "paths %u rays %zu tokens %zu pixels %u items %u\n", npaths, t.ray_start.size()-1, t.tok.size(), npix, nitems);
    Stats S;
    // one wave consumes the whole item stream (statistically like any wave)
    int st[64]; uint32_t path[64], ray[64], pos[64], end[64], bleft[64], samp[64], pix[64];
    for (int l = 0; l < 64; l++) st[l] = NEED;
    uint32_t qnext = 0, res_base = 0, res_cnt = 0; bool qdone = false;
    auto tokat = [&](int l) { return t.tok[pos[l]]; };
    auto start_ray = [&](int l) { uint32_t r = t.path_start[path[l]] + ray[l]; pos[l] = t.ray_start[r]; end[l] = t.ray_start[r + 1]; S.rays++; };
    for (;;) {
        S.iters++;
        for (;;) {
            uint64_t need = 0; for (int l = 0; l < 64; l++) if (st[l] == NEED) need |= 1ull << l;
            while (need && !qdone) {
                if (res_cnt == 0) { if (qnext >= nitems) { qdone = true; break; } res_base = qnext; res_cnt = min<uint32_t>(p.claim, nitems - qnext); qnext += res_cnt; }
                for (int l = 0; l < 64 && res_cnt; l++) if (need >> l & 1) {
                    uint32_t q = res_base++; res_cnt--; need &= ~(1ull << l);
                    pix[l] = q / cpp; samp[l] = (q % cpp) * p.chunk; bleft[l] = p.chunk; st[l] = CAM;
                }
            }
            int ncam = 0, ntrace = 0;
            for (int l = 0; l < 64; l++) { ncam += st[l] == CAM; ntrace += st[l] == TRACE; }
            if (ncam && (ncam >= p.adv_min || ntrace == 0 || qdone)) {
                int wmax = 0; double wsum = 0;
                for (int l = 0; l < 64; l++) if (st[l] == CAM) { path[l] = pix[l] * p.spp + samp[l]; ray[l] = 0; start_ray(l); st[l] = TRACE;
                    wmax = max<int>(wmax, t.wit[path[l]]); wsum += t.wit[path[l]]; }
                S.adv++; S.adv_lanes += ncam; S.w_max += wmax; S.w_sum += wsum; S.w_coop += coop_rounds(t, path, st, ncam, 2);
            }
            bool anyneed = false; for (int l = 0; l < 64; l++) anyneed |= st[l] == NEED;
            if (qdone || !anyneed) break;
        }
        for (int l = 0; l < 64; l++) if (st[l] == NEED) st[l] = DONE;
        bool any = false; for (int l = 0; l < 64; l++) any |= st[l] == TRACE || st[l] == SHADE;
        if (!any) break;
        int alive = 0; for (int l = 0; l < 64; l++) alive += st[l] != DONE;
        for (;;) {
            int ntr = 0, nlm = 0;
            for (int l = 0; l < 64; l++) if (st[l] == TRACE && pos[l] < end[l]) { ntr++; if (tokat(l) != 0) nlm++; }
            if (ntr == 0) break;
            if (alive - ntr >= p.shade_batch) break;
            bool leaf_pass = nlm == ntr || nlm >= p.leaf_batch;
            if (!leaf_pass) {
                S.node_passes++; S.node_pass_lanes += ntr;
                for (int s = 0; s < p.steps; s++) {
                    if (p.exit_k && s > 0) { int c = 0; for (int l = 0; l < 64; l++) c += st[l] == TRACE && pos[l] < end[l] && tokat(l) == 0; if (c < p.exit_k) { S.early++; break; } }
                    int act = 0;
                    for (int l = 0; l < 64; l++) if (st[l] == TRACE && pos[l] < end[l] && tokat(l) == 0) { act++; pos[l]++; S.nodes++; }
                    if (act) { S.wsteps++; S.step_lanes += act; }
                }
            } else {
                S.leaf_passes++; S.leaf_lanes += nlm;
                bool sq1 = false, sq2 = false, dv1 = false, dv2 = false, both = false, anysq = false, any2nd = false;
                for (int l = 0; l < 64; l++) if (st[l] == TRACE && pos[l] < end[l] && tokat(l) != 0) {
                    int tk = tokat(l), o1, o2 = -1;
                    if (tk >= 32) { o1 = (tk - 32) / 4; o2 = (tk - 32) % 4; S.spheres += 2; } else { o1 = tk - 16; S.spheres += 1; }
                    bool n1 = o1 > 0, n2 = o2 > 0;
                    sq1 |= n1; sq2 |= n2; dv1 |= o1 == 1 || o1 == 2; dv2 |= o2 == 1 || o2 == 2;
                    both |= n1 && n2; anysq |= n1 || n2;
                    int k2 = (o1 == 1 || o1 == 2) + (o2 == 1 || o2 == 2); any2nd |= k2 > 0;
                    pos[l]++;
                }
                S.b_sq1 += sq1; S.b_sq2 += sq2; S.b_dv1 += dv1; S.b_dv2 += dv2; S.b_both += both; S.b_any += anysq; S.b_2nd += any2nd;
            }
        }
        int ns = 0;
        for (int l = 0; l < 64; l++) if (st[l] == TRACE && pos[l] >= end[l]) { st[l] = SHADE; }
        { int umax = 0, nu = 0; double usum = 0;
          for (int l = 0; l < 64; l++) if (st[l] == SHADE) { int u = t.uit[t.path_start[path[l]] + ray[l]]; if (u) { nu++; umax = max(umax, u); usum += u; } }
          if (nu) { S.u_passes++; S.u_lanes += nu; S.u_max += umax; S.u_sum += usum; } }
        for (int l = 0; l < 64; l++) if (st[l] == SHADE) {
            ns++;
            uint32_t nr = t.path_start[path[l] + 1] - t.path_start[path[l]];
            if (ray[l] + 1 < nr) { ray[l]++; start_ray(l); st[l] = TRACE; }
            else { bleft[l]--; if (bleft[l] == 0) st[l] = NEED; else { samp[l]++; st[l] = CAM; } }
        }
        if (ns) { S.shade_passes++; S.shade_lanes += ns; }
    }
    double R = S.rays;
    printf("shade_batch %d leaf_batch %d steps %d | rays %.0f nodes/ray %.2f sph/ray %.2f\n", p.shade_batch, p.leaf_batch, p.steps, R, S.nodes / R, S.spheres / R);
    printf("per ray: iters %.4f node_passes %.4f (%.1f lanes) wsteps %.4f (%.1f lanes) leaf_passes %.4f (%.1f lanes) shade %.4f (%.1f lanes) adv %.4f (%.1f lanes)\n",
           S.iters / R, S.node_passes / R, S.node_pass_lanes / S.node_passes, S.wsteps / R, S.step_lanes / S.wsteps, S.leaf_passes / R,
           S.leaf_lanes / S.leaf_passes, S.shade_passes / R, S.shade_lanes / S.shade_passes, S.adv / R, S.adv_lanes / S.adv);
    printf("early node-pass exits per ray %.4f\n", S.early / R);
    printf("camera disk loop: per advance %.2f wave iterations (lane mean %.2f)\n", S.w_max / S.adv, S.w_sum / S.adv_lanes);
    printf("unit-sphere loop: %.3f of shade passes, %.1f lanes, %.2f wave iterations (lane mean %.2f)\n", S.u_passes / S.shade_passes,
           S.u_lanes / S.u_passes, S.u_max / S.u_passes, S.u_sum / S.u_lanes);
    printf("leaf pass blocks: sqrt1 %.3f sqrt2 %.3f div2nd1 %.3f div2nd2 %.3f | merged: any %.3f both %.3f any2nd %.3f\n",
           S.b_sq1 / S.leaf_passes, S.b_sq2 / S.leaf_passes, S.b_dv1 / S.leaf_passes, S.b_dv2 / S.leaf_passes,
           S.b_any / S.leaf_passes, S.b_both / S.leaf_passes, S.b_2nd / S.leaf_passes);
    const double CN = getenv("CN") ? atof(getenv("CN")) : 60, CL = getenv("CL") ? atof(getenv("CL")) : 400,
                 CS = getenv("CS") ? atof(getenv("CS")) : 3500, CA = getenv("CA") ? atof(getenv("CA")) : 3000;
    const double cyc = S.wsteps * CN + S.leaf_passes * CL + S.shade_passes * CS + S.adv * CA + S.iters * 60 + S.node_passes * 30;
    printf("model cycles/ray %.1f  (node %.1f leaf %.1f shade %.1f adv %.1f head %.1f)\n", cyc / R, S.wsteps * CN / R, S.leaf_passes * CL / R,
           S.shade_passes * CS / R, S.adv * CA / R, (S.iters * 60 + S.node_passes * 30) / R);
}
