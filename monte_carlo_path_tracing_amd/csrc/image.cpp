// Tone mapping and BMP output of the render driver (main.cpp:582-596).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "mcpt_internal.h"

extern "C" {

// RadianceRGB::tone_mapping (RadianceRGB.cpp:51-67): clamp(floor(255 * (L/max)^gamma + 0.5)),
// with x86's out-of-range float->int conversion (INT_MIN, hence 0) for NaN/huge values.
int mcpt_tone_map(const double* rgb, int32_t width, int32_t height, double maxr, double gamma, uint8_t* out) {
    if (!rgb || !out || width <= 0 || height <= 0) {
        mcpt::set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    const double A = std::pow(maxr, -gamma);
    const size_t n = 3ull * width * height;
    for (size_t k = 0; k < n; k++) {
        const double r = A * std::pow(rgb[k], gamma);
        const double x = std::floor(r * 255 + 0.5);
        const int v = (x >= -2147483648.0 && x < 2147483648.0) ? static_cast<int>(x) : static_cast<int>(0x80000000u);
        out[k] = static_cast<uint8_t>(v > 255 ? 255 : (v < 0 ? 0 : v));
    }
    return MCPT_OK;
}

// The layout EasyX saveimage produced for test.bmp: BITMAPINFOHEADER, 32 bpp, BI_RGB,
// bottom-up rows, 3780 px/m, pixels B G R 0 (main.cpp:585 packs BGR(RGB(r,g,b))).
int mcpt_write_bmp(const char* path, const uint8_t* rgb8, int32_t width, int32_t height) {
    if (!path || !rgb8 || width <= 0 || height <= 0) {
        mcpt::set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    const uint32_t img = 4u * width * height;
    uint8_t h[54];
    std::memset(h, 0, sizeof h);
    auto put32 = [&](int off, uint32_t v) { std::memcpy(h + off, &v, 4); };
    auto put16 = [&](int off, uint16_t v) { std::memcpy(h + off, &v, 2); };
    h[0] = 'B';
    h[1] = 'M';
    put32(2, 54 + img);
    put32(10, 54);
    put32(14, 40);
    put32(18, static_cast<uint32_t>(width));
    put32(22, static_cast<uint32_t>(height));
    put16(26, 1);
    put16(28, 32);
    put32(38, 3780);
    put32(42, 3780);
    std::vector<uint8_t> px(img);
    for (int i = 0; i < height; i++) {
        const int row = height - 1 - i;  // bottom-up
        for (int j = 0; j < width; j++) {
            const uint8_t* s = rgb8 + 3 * ((size_t)i * width + j);
            uint8_t* d = px.data() + 4 * ((size_t)row * width + j);
            d[0] = s[2];
            d[1] = s[1];
            d[2] = s[0];
            d[3] = 0;
        }
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        mcpt::set_error("cannot write %s", path);
        return MCPT_E_IO;
    }
    const bool ok = std::fwrite(h, 1, 54, f) == 54 && std::fwrite(px.data(), 1, img, f) == img;
    std::fclose(f);
    if (!ok) {
        mcpt::set_error("short write %s", path);
        return MCPT_E_IO;
    }
    return MCPT_OK;
}

}  // extern "C"
