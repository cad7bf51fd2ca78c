// image_io.h — PNG / Radiance HDR decode and encode for the host front-end (see image_io.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace rth {

struct Image8 {
    int width = 0, height = 0, channels = 0;
    std::vector<uint8_t> data;
};
struct ImageF {
    int width = 0, height = 0;
    std::vector<float> data;  // RGB
};

bool decode_png(const std::string& path, Image8& img, std::string& err);
bool encode_png(const std::string& path, int w, int h, int channels, const uint8_t* rgb, std::string& err);
bool decode_hdr(const std::string& path, ImageF& img, std::string& err);
// JPEG (baseline + progressive, 8-bit; jpeg_decode.cpp)
bool decode_jpeg(const std::string& path, Image8& img, std::string& err);
bool decode_jpeg_mem(const uint8_t* data, size_t n, Image8& img, std::string& err);
// PNG or JPEG by content (stbi_load's format sniffing for the formats RTBase scenes use)
bool decode_ldr(const std::string& path, Image8& img, std::string& err);
bool encode_hdr(const std::string& path, int w, int h, const float* rgb, std::string& err);

}  // namespace rth
