// image.hpp — Image<T>, Color and device images of the C++ host (the reference's
// src/lib/image.rs and src/lib/color.rs, host side), plus the GPU context they live on.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../eray_hip.h"

namespace eray {

// color.rs:12-22 (#[repr(C)] r, g, b f32)
struct Color {
    float r = 0.0f, g = 0.0f, b = 0.0f;
    Color() = default;
    Color(float r_, float g_, float b_) : r(r_), g(g_), b(b_) {}
    bool operator==(const Color& o) const { return r == o.r && g == o.g && b == o.b; }
    // color.rs:31-37: (c * 255.) as u8 per channel (saturating, NaN -> 0)
    void as_bytes(uint8_t out[3]) const;
};

// image.rs:8-74 — host image, row-major, y = 0 is the bottom row of the viewport
template <typename T>
struct Image {
    uint32_t width = 0, height = 0;
    std::vector<T> pixels;

    Image() = default;
    Image(uint32_t w, uint32_t h, T fill) : width(w), height(h), pixels((size_t)w * h, fill) {}
    // image.rs:36-38
    const T& mod_get(uint32_t x, uint32_t y) const { return pixels[(size_t)(y % height) * width + (x % width)]; }
    // image.rs:41-43 (panics out of range: std::out_of_range here)
    void set(uint32_t x, uint32_t y, const T& v) { pixels.at((size_t)y * width + x) = v; }
    bool operator==(const Image& o) const { return width == o.width && height == o.height && pixels == o.pixels; }
};

// The reference's debug side-effect files — rgb.ppm written by every rgb node run (rgb.rs:96)
// and color.ppm by Material::update in debug builds (material.rs:41-50) — into the working
// directory.  On by default in builds without NDEBUG (as a `cargo run` debug build), settable.
bool debug_dumps();
void set_debug_dumps(bool on);

// image.rs:48-74 (Image<Color>::save_as_ppm): "P6 {w} {h} 255\n" + rows y = h-1 .. 0
std::vector<uint8_t> ppm_bytes(const Image<Color>& image);
void save_as_ppm(const Image<Color>& image, const std::string& path);

// The GPU context the host objects use (one per GPU / rank; eray_ctx of the C-ABI).
class Device {
public:
    explicit Device(int gpu = 0);
    ~Device();
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;
    eray_ctx* ctx() const { return ctx_; }
    // throws eray::Failure with the C-ABI status and message when status != 0
    void check(int status) const;
    // The calling thread's current device (created on GPU 0 on first use).
    static Device& current();
    static void set_current(std::shared_ptr<Device> device);

private:
    eray_ctx* ctx_ = nullptr;
};

struct Failure : std::runtime_error {
    int status;
    Failure(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

// A device allocation on the current device (shared, freed with the last owner).
class DeviceBuffer {
public:
    explicit DeviceBuffer(size_t bytes);
    ~DeviceBuffer();
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    void* data() const { return ptr_; }
    size_t size() const { return bytes_; }

private:
    void* ptr_ = nullptr;
    size_t bytes_ = 0;
};

// A device image of T = float (IValue) or Color (IColor): what the node operators produce.
template <typename T>
struct DeviceImage {
    uint32_t width = 0, height = 0;
    std::shared_ptr<DeviceBuffer> buffer;

    DeviceImage() = default;
    DeviceImage(uint32_t w, uint32_t h)
        : width(w), height(h), buffer(std::make_shared<DeviceBuffer>(sizeof(T) * (size_t)w * h)) {}
    T* data() const { return buffer ? static_cast<T*>(buffer->data()) : nullptr; }
    eray_image view() const { return eray_image{reinterpret_cast<const float*>(data()), width, height}; }
    Image<T> to_host() const;
    static DeviceImage from_host(const Image<T>& image);
    // the same buffer (shared, as the reference's value clones are never mutated in place)
    bool operator==(const DeviceImage& o) const { return buffer == o.buffer && width == o.width && height == o.height; }
};

extern template struct DeviceImage<float>;
extern template struct DeviceImage<Color>;

}  // namespace eray
