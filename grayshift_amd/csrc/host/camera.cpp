// camera.cpp — Camera::new (camera.rs:39-98) and Camera::render (camera.rs:100-121).
// render() replaces the rayon pixel loop (camera.rs:105-114) and the output stage
// (:101-103,116-118) with one gs_render_ppm call: bytes and text come from the device.
#include <cstring>
#include <sstream>

#include "world.hpp"

namespace grayshift {

Camera::Camera(double aspect_ratio, int32_t image_width, SampleSettings s, uint32_t max_depth, double v_fov,
               Vec3 look_from, Vec3 look_at, Vec3 vup, double defocus_angle, double focus_distance,
               Background background)
    : bg(background) {
    const int32_t image_height = (int32_t)((double)image_width / aspect_ratio);  // `as i32`
    const double theta = v_fov / 180.0 * PI;
    const double h = std::tan(theta / 2.0);
    const double viewport_height = 2.0 * h * focus_distance;
    const double viewport_width = viewport_height * ((double)image_width / (double)image_height);
    const Vec3 w = (look_from - look_at).unit();
    const Vec3 u = vup.cross(w).unit();
    const Vec3 v = w.cross(u);
    const Vec3 viewport_u = viewport_width * u;
    const Vec3 viewport_v = viewport_height * -v;
    const Vec3 pixel_delta_u = viewport_u / (double)image_width;
    const Vec3 pixel_delta_v = viewport_v / (double)image_height;
    const Vec3 viewport_upper_left = look_from - focus_distance * w - viewport_u / 2.0 - viewport_v / 2.0;
    const Vec3 starting_pixel_pos = viewport_upper_left + 0.5 * (pixel_delta_u + pixel_delta_v);
    const double defocus_radius = focus_distance * std::tan((defocus_angle / 2.0) / 180.0 * PI);
    const Vec3 defocus_disk_u = u * defocus_radius;
    const Vec3 defocus_disk_v = v * defocus_radius;

    std::memset(&cam, 0, sizeof(cam));
    cam.image_width = image_width;
    cam.image_height = image_height;
    cam.max_depth = max_depth;
    look_from.store(cam.center);
    starting_pixel_pos.store(cam.starting_pixel_pos);
    pixel_delta_u.store(cam.pixel_delta_u);
    pixel_delta_v.store(cam.pixel_delta_v);
    cam.defocus_angle = defocus_angle;
    defocus_disk_u.store(cam.defocus_disk_u);
    defocus_disk_v.store(cam.defocus_disk_v);
    ss.confidence = s.confidence;
    ss.tolerance = s.tolerance;
    ss.batch_size = s.batch_size;
    ss.max_samples = s.max_samples;
}

static void check(gs_status st) {
    if (st != GS_OK) throw std::runtime_error(std::string("gs_render failed: ") + gs_last_error());
}

void Camera::render_linear(const Hittable& world, float* out_rgb, gs_stats* stats, uint64_t seed) const {
    auto fs = flatten_world(world, bg);
    check(gs_render(&fs->view, &cam, &ss, seed, out_rgb, stats));
}

std::string Camera::render_ppm(const Hittable& world, gs_stats* stats, uint64_t seed) const {
    auto fs = flatten_world(world, bg);
    const int64_t cap = gs_ppm_max_bytes(cam.image_width, cam.image_height);
    if (cap < 0) throw std::runtime_error("bad image size");
    std::string text((size_t)cap, '\0');
    int64_t len = 0;
    check(gs_render_ppm(&fs->view, &cam, &ss, seed, &text[0], cap, &len, stats));
    text.resize((size_t)len);
    return text;
}

// The whole of camera.rs:100-121: the PPM text (header, then write_color per pixel of
// the f64 colour) is formatted on the device and written here with one call.
void Camera::render(const Hittable& world, std::ostream& image_file, uint64_t seed) const {
    const std::string text = render_ppm(world, nullptr, seed);
    image_file.write(text.data(), (std::streamsize)text.size());
    if (!image_file) throw std::runtime_error("PPM write failed");
}

int32_t color_byte(double c) {  // color.rs:8-28
    double g = c > 0.0 ? std::sqrt(c) : 0.0;  // linear_to_gamma
    double cl = g;                             // INTENSITY.clamp: Rust f64::clamp, NaN passes through
    if (cl < 0.000) cl = 0.000;
    if (cl > 0.999) cl = 0.999;
    double b = 256.0 * cl;
    if (std::isnan(b)) return 0;  // `as i32` saturates, NaN -> 0
    return (int32_t)b;
}

void write_ppm(std::ostream& os, int32_t w, int32_t h, const float* rgb) {  // camera.rs:101-103,116-118
    os << "P3\n" << w << " " << h << "\n255\n";
    const size_t n = (size_t)w * (size_t)h;
    for (size_t k = 0; k < n; k++)
        os << color_byte(rgb[3 * k]) << " " << color_byte(rgb[3 * k + 1]) << " " << color_byte(rgb[3 * k + 2]) << "\n";
}

}  // namespace grayshift
