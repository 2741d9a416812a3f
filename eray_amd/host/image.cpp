// image.cpp — Color / Image / PPM writer and the device plumbing of the C++ host.
#include "eray/image.hpp"

#include <cmath>
#include <cstdio>
#include <fstream>
#include <mutex>

namespace eray {

namespace {
// Rust's `f as u8`: saturating, NaN -> 0 (color.rs:31-37)
uint8_t sat_u8(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)f;
}
}  // namespace

void Color::as_bytes(uint8_t out[3]) const {
    out[0] = sat_u8(r * 255.0f);
    out[1] = sat_u8(g * 255.0f);
    out[2] = sat_u8(b * 255.0f);
}

std::vector<uint8_t> ppm_bytes(const Image<Color>& image) {
    char header[64];
    size_t len = 0;
    if (eray_ppm_header(image.width, image.height, header, sizeof header, &len) != ERAY_OK)
        throw Failure(ERAY_E_INVALID_ARGUMENT, "ppm header");
    std::vector<uint8_t> out(header, header + len);
    out.reserve(len + (size_t)image.width * image.height * 3);
    for (uint32_t k = 0; k < image.height; ++k) {  // image.rs:59-72: rows y = h-1 .. 0
        const uint32_t y = image.height - 1 - k;
        for (uint32_t x = 0; x < image.width; ++x) {
            uint8_t b[3];
            image.pixels[(size_t)y * image.width + x].as_bytes(b);
            out.insert(out.end(), b, b + 3);
        }
    }
    return out;
}

namespace {
#ifdef NDEBUG
bool g_debug_dumps = false;
#else
bool g_debug_dumps = true;
#endif
}  // namespace
bool debug_dumps() { return g_debug_dumps; }
void set_debug_dumps(bool on) { g_debug_dumps = on; }

void save_as_ppm(const Image<Color>& image, const std::string& path) {
    const std::vector<uint8_t> bytes = ppm_bytes(image);
    std::ofstream f(path, std::ios::binary);
    if (!f) throw Failure(ERAY_E_IO, "cannot open " + path);
    f.write(reinterpret_cast<const char*>(bytes.data()), (std::streamsize)bytes.size());
    if (!f) throw Failure(ERAY_E_IO, "cannot write " + path);
}

// ---------------------------------------------------------------------------- Device -----
Device::Device(int gpu) {
    eray_ctx* c = nullptr;
    const int st = eray_ctx_create(gpu, &c);
    if (st != ERAY_OK) throw Failure(st, eray_last_error(nullptr));
    ctx_ = c;
}

Device::~Device() {
    if (ctx_) eray_ctx_destroy(ctx_);
}

void Device::check(int status) const {
    if (status != ERAY_OK) throw Failure(status, eray_last_error(ctx_));
}

namespace {
thread_local std::shared_ptr<Device> t_current;
}

Device& Device::current() {
    if (!t_current) t_current = std::make_shared<Device>(0);
    return *t_current;
}

void Device::set_current(std::shared_ptr<Device> device) { t_current = std::move(device); }

DeviceBuffer::DeviceBuffer(size_t bytes) : bytes_(bytes) {
    Device& d = Device::current();
    d.check(eray_device_alloc(d.ctx(), bytes ? bytes : 1, &ptr_));
}

DeviceBuffer::~DeviceBuffer() {
    if (ptr_) eray_device_free(Device::current().ctx(), ptr_);
}

template <typename T>
Image<T> DeviceImage<T>::to_host() const {
    Image<T> img(width, height, T{});
    if (!img.pixels.empty()) {
        Device& d = Device::current();
        d.check(eray_copy_to_host(d.ctx(), img.pixels.data(), data(), sizeof(T) * img.pixels.size()));
    }
    return img;
}

template <typename T>
DeviceImage<T> DeviceImage<T>::from_host(const Image<T>& image) {
    DeviceImage<T> d(image.width, image.height);
    if (!image.pixels.empty()) {
        Device& dev = Device::current();
        dev.check(eray_copy_to_device(dev.ctx(), d.data(), image.pixels.data(), sizeof(T) * image.pixels.size()));
    }
    return d;
}

template struct DeviceImage<float>;
template struct DeviceImage<Color>;

}  // namespace eray
