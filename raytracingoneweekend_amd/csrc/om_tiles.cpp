// om_tiles.cpp — conservative per-tile primary-ray candidate lists (see om_tiles.h).
//
// A primary ray of pixel (i, j) starts at a lens point L = O + off (|off| <= lens_radius,
// off in the u/v plane) and passes through the focus-plane point
// P = llc + u H + v V with u = (i + r)/(W-1), v = 1 - (j + r')/(H-1), r, r' in [0, 1]
// (camera.rs:60-74, render_thread.rs:183-192).  A point X is reached through the focus
// plane at P_L = P_O + off (1 - s), where P_O is X's projection from O and s = the ratio
// ((llc - O).n) / ((X - O).n) with n = H x V.  So over the lens the projection of X moves
// by at most R |1 - s| in the focus plane.  For a box in front of the camera the
// projection from O is the hull of the corner projections and |1 - s| peaks at a corner,
// which bounds the (u, v) footprint of every ray that can touch the box.  Boxes wholly
// behind the lens plane are never reached; boxes straddling it go to every tile.
// Everything is evaluated in double with a 3-pixel margin, far beyond the f32 rounding
// of the kernel's ray set-up.
#include "om_tiles.h"

#include <algorithm>
#include <cmath>

namespace omt {
namespace {

struct D3 { double x, y, z; };
D3 d3(const float* p) { return D3{p[0], p[1], p[2]}; }
D3 sub(D3 a, D3 b) { return D3{a.x - b.x, a.y - b.y, a.z - b.z}; }
D3 add(D3 a, D3 b) { return D3{a.x + b.x, a.y + b.y, a.z + b.z}; }
D3 scl(D3 a, double s) { return D3{a.x * s, a.y * s, a.z * s}; }
double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 cross(D3 a, D3 b) { return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
bool finite3(D3 a) { return std::isfinite(a.x) && std::isfinite(a.y) && std::isfinite(a.z); }

}  // namespace

bool build(const std::vector<float>& srec_box, const om_camera& cam, uint32_t W, uint32_t H, TileLists& out) {
    out = TileLists{};
    const size_t nrec = srec_box.size() / 6;
    if (W < 2 || H < 2 || nrec > 65535u) return false;
    const D3 O = d3(cam.origin), Hh = d3(cam.horizontal), Vv = d3(cam.vertical), llc = d3(cam.lower_left_corner);
    const double R = std::fabs((double)cam.lens_radius);
    const D3 n = cross(Hh, Vv);
    const double hh = dot(Hh, Hh), vv = dot(Vv, Vv), num = dot(sub(llc, O), n);
    if (!finite3(O) || !finite3(Hh) || !finite3(Vv) || !finite3(llc) || !std::isfinite(R) || !(hh > 0) || !(vv > 0) ||
        !(std::fabs(num) > 0))
        return false;
    const uint32_t tx = (W + 7u) / 8u, ty = (H + 7u) / 8u, ntiles = tx * ty;
    const double wm1 = (double)(W - 1u), hm1 = (double)(H - 1u);
    struct Rect { uint32_t x0, x1, y0, y1; };
    std::vector<Rect> rect(nrec);
    // Early-out bound (traced_tiles<true>): a primary ray starts at a lens point
    // L (|L - O| <= R) with a unit direction, so it reaches the box no earlier than
    // t = dist(O, box) - R.  Margins: 1e-5 relative + 1e-4 for the f32 ray set-up and root.
    out.tnear.assign(nrec, 0.0f);
    for (size_t r = 0; r < nrec; ++r) {
        const float* b = &srec_box[6 * r];
        double dd = 0.0;
        const double o[3] = {O.x, O.y, O.z};
        for (int a = 0; a < 3; ++a) {
            const double e = std::max({(double)b[a] - o[a], 0.0, o[a] - (double)b[3 + a]});
            dd += e * e;
        }
        const double t = (std::sqrt(dd) - R) * (1.0 - 1e-5) - 1e-4;
        float f = t > 0.0 ? (float)t : 0.0f;
        if ((double)f > t) f = std::nextafter(f, -INFINITY);
        out.tnear[r] = std::isfinite(f) && f > 0.0f ? f : 0.0f;
    }
    std::vector<uint32_t> cnt(ntiles, 0u);
    for (size_t r = 0; r < nrec; ++r) {
        const float* b = &srec_box[6 * r];
        double a0 = INFINITY, a1 = -INFINITY, b0 = INFINITY, b1 = -INFINITY, k = 0.0;
        bool all = false;
        // a box wholly behind the lens plane (through O, normal n; every lens point lies on
        // it) is never reached: a ray's points X = L + t (P - L), t >= tmin > 0, have
        // (X - O).n of num's sign.  Margin: 1e-6 relative + 1e-4 world units (f32 origins).
        int behind = 0;
        const double nl = std::sqrt(dot(n, n));
        for (int c = 0; c < 8; ++c) {
            const D3 X{(c & 1) ? b[3] : b[0], (c & 2) ? b[4] : b[1], (c & 4) ? b[5] : b[2]};
            const D3 dX = sub(X, O);
            const double ahead = dot(dX, n) / nl * (num > 0 ? 1.0 : -1.0);     // signed distance in front
            behind += ahead < -(1e-6 * std::sqrt(dot(dX, dX)) + 1e-4) ? 1 : 0;
        }
        if (behind == 8) { rect[r] = Rect{1u, 0u, 1u, 0u}; continue; }
        for (int c = 0; c < 8 && !all; ++c) {
            const D3 X{(c & 1) ? b[3] : b[0], (c & 2) ? b[4] : b[1], (c & 4) ? b[5] : b[2]};
            const D3 dX = sub(X, O);
            const double den = dot(dX, n);
            // the corner must lie clearly on the focus plane's side of the camera
            if (!(den * num > 0.0) || std::fabs(den) < 1e-9 * std::sqrt(dot(dX, dX) * dot(n, n))) { all = true; break; }
            const double s = num / den;
            const D3 Pm = sub(add(O, scl(dX, s)), llc);
            const double a = dot(Pm, Hh) / hh, bb = dot(Pm, Vv) / vv;
            a0 = std::min(a0, a); a1 = std::max(a1, a);
            b0 = std::min(b0, bb); b1 = std::max(b1, bb);
            k = std::max(k, std::fabs(1.0 - s));
        }
        int64_t i0 = 0, i1 = (int64_t)W - 1, j0 = 0, j1 = (int64_t)H - 1;
        if (!all) {
            const double da = R * k / std::sqrt(hh), db = R * k / std::sqrt(vv);
            a0 -= da; a1 += da; b0 -= db; b1 += db;
            if (!std::isfinite(a0 + a1 + b0 + b1)) {
                all = true;
            } else {
                const double fi0 = std::floor(a0 * wm1) - 3.0, fi1 = std::ceil(a1 * wm1) + 2.0;
                const double fj0 = std::floor((1.0 - b1) * hm1) - 3.0, fj1 = std::ceil((1.0 - b0) * hm1) + 2.0;
                i0 = (int64_t)std::max(fi0, -1.0); i1 = (int64_t)std::min(fi1, (double)W);
                j0 = (int64_t)std::max(fj0, -1.0); j1 = (int64_t)std::min(fj1, (double)H);
                i0 = std::max<int64_t>(i0, 0); j0 = std::max<int64_t>(j0, 0);
                i1 = std::min<int64_t>(i1, (int64_t)W - 1); j1 = std::min<int64_t>(j1, (int64_t)H - 1);
            }
        }
        if (all) { i0 = 0; i1 = W - 1; j0 = 0; j1 = H - 1; }
        if (i0 > i1 || j0 > j1) { rect[r] = Rect{1u, 0u, 1u, 0u}; continue; }
        rect[r] = Rect{(uint32_t)(i0 / 8), (uint32_t)(i1 / 8), (uint32_t)(j0 / 8), (uint32_t)(j1 / 8)};
        for (uint32_t y = rect[r].y0; y <= rect[r].y1; ++y)
            for (uint32_t x = rect[r].x0; x <= rect[r].x1; ++x) cnt[y * tx + x]++;
    }
    out.off.assign(ntiles + 1u, 0u);
    uint64_t total = 0;
    double seen = 0.0;
    for (uint32_t t = 0; t < ntiles; ++t) {
        out.off[t] = (uint32_t)total;
        total += cnt[t];
        const uint32_t pw = std::min(8u, W - (t % tx) * 8u), ph = std::min(8u, H - (t / tx) * 8u);
        seen += (double)cnt[t] * pw * ph;
    }
    if (total > (1ull << 28)) { out = TileLists{}; return false; }
    out.off[ntiles] = (uint32_t)total;
    out.avg_per_pixel = seen / ((double)W * H);
    out.idx.resize(total);
    std::vector<uint32_t> pos(out.off.begin(), out.off.end() - 1);
    for (size_t r = 0; r < nrec; ++r) {                                    // ascending record order per tile
        const Rect& q = rect[r];
        for (uint32_t y = q.y0; y <= q.y1 && q.x0 <= q.x1; ++y)
            for (uint32_t x = q.x0; x <= q.x1; ++x) out.idx[pos[y * tx + x]++] = (uint16_t)r;
    }
    for (uint32_t t = 0; t < ntiles; ++t)                                  // nearest first (the early-out)
        std::stable_sort(out.idx.begin() + out.off[t], out.idx.begin() + out.off[t + 1],
                         [&](uint16_t a, uint16_t b) { return out.tnear[a] < out.tnear[b]; });
    return true;
}

}  // namespace omt
