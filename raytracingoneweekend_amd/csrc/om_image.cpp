// om_image.cpp — headless image writers for the display views (the reference saves the
// SDL surface with F12 as <unix time>.bmp, main.rs:473-476).
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/ottomarcher.h"

namespace {

void le16(unsigned char* p, uint32_t v) { p[0] = (unsigned char)v; p[1] = (unsigned char)(v >> 8); }
void le32(unsigned char* p, uint32_t v) { for (int i = 0; i < 4; ++i) p[i] = (unsigned char)(v >> (8 * i)); }

bool valid(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h) {
    return path && rgb && w > 0 && h > 0 && (uint64_t)w * h <= 0x3FFFFFFFull;
}

}  // namespace

extern "C" {

// 24-bit BI_RGB bitmap: 14-byte file header + 40-byte BITMAPINFOHEADER, rows bottom-up in
// BGR order, each row padded to a multiple of 4 bytes.
om_status om_write_bmp(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h) {
    if (!valid(path, rgb, w, h)) return OM_ERR_INVALID;
    const uint32_t stride = (3u * w + 3u) & ~3u;
    const uint64_t image = (uint64_t)stride * h;
    if (image + 54u > 0xFFFFFFFFull) return OM_ERR_INVALID;
    unsigned char hdr[54];
    std::memset(hdr, 0, sizeof(hdr));
    hdr[0] = 'B'; hdr[1] = 'M';
    le32(hdr + 2, (uint32_t)(image + 54u));
    le32(hdr + 10, 54u);
    le32(hdr + 14, 40u);
    le32(hdr + 18, w);
    le32(hdr + 22, h);
    le16(hdr + 26, 1u);
    le16(hdr + 28, 24u);
    le32(hdr + 34, (uint32_t)image);
    FILE* f = std::fopen(path, "wb");
    if (!f) return OM_ERR_INVALID;
    bool ok = std::fwrite(hdr, 1, sizeof(hdr), f) == sizeof(hdr);
    std::vector<unsigned char> row(stride, 0);
    for (uint32_t y = h; ok && y-- > 0;) {
        const uint8_t* src = rgb + (size_t)y * w * 3u;
        for (uint32_t x = 0; x < w; ++x) {
            row[3 * x + 0] = src[3 * x + 2];
            row[3 * x + 1] = src[3 * x + 1];
            row[3 * x + 2] = src[3 * x + 0];
        }
        ok = std::fwrite(row.data(), 1, stride, f) == stride;
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? OM_OK : OM_ERR_INVALID;
}

// Binary PPM (P6, maxval 255), rows top-down in RGB order.
om_status om_write_ppm(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h) {
    if (!valid(path, rgb, w, h)) return OM_ERR_INVALID;
    FILE* f = std::fopen(path, "wb");
    if (!f) return OM_ERR_INVALID;
    bool ok = std::fprintf(f, "P6\n%u %u\n255\n", w, h) > 0;
    const size_t n = (size_t)w * h * 3u;
    ok = ok && std::fwrite(rgb, 1, n, f) == n;
    ok = (std::fclose(f) == 0) && ok;
    return ok ? OM_OK : OM_ERR_INVALID;
}

}  // extern "C"
