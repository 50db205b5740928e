// misc.cpp — G_Buffer seeds (rt/screen.cuh:34-45) and the PNG writer that
// replaces lodepng::encode in save_render (rt/save_render.cuh:18-23).
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "rt_host.h"

namespace rt_host {

// std::mt19937 generator; uniform_int_distribution<uint32_t>(0, UINT32_MAX):
// the full-range distribution returns the engine's raw 32-bit words.
void mt19937_seeds(uint32_t *out, size_t count, uint64_t skip)
{
    std::mt19937 generator;
    std::uniform_int_distribution<uint32_t> distribution(0, UINT32_MAX);
    generator.discard(skip);
    for (size_t i = 0; i < count; ++i) out[i] = distribution(generator);
}

namespace {
uint32_t crc_table[256];
bool crc_ready = false;
void crc_init()
{
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
    crc_ready = true;
}
uint32_t crc32(const uint8_t *b, size_t n, uint32_t c = 0xffffffffu)
{
    for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ b[i]) & 0xff] ^ (c >> 8);
    return c;
}
void be32(std::vector<uint8_t> &v, uint32_t x)
{
    v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
}
void chunk(FILE *f, const char *type, const std::vector<uint8_t> &data)
{
    std::vector<uint8_t> buf;
    be32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    uint32_t c = crc32(buf.data() + 4, buf.size() - 4) ^ 0xffffffffu;
    be32(buf, c);
    fwrite(buf.data(), 1, buf.size(), f);
}
} // namespace

// RGBA8, rows written top to bottom in the order given; zlib "stored" blocks
int write_png(const char *path, const uint8_t *rgba, int w, int h)
{
    if (!crc_ready) crc_init();
    FILE *f = fopen(path, "wb");
    if (!f) {
        rt_set_error("cannot write %s", path);
        return RT_E_IO;
    }
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    fwrite(sig, 1, 8, f);
    std::vector<uint8_t> ihdr;
    be32(ihdr, (uint32_t)w);
    be32(ihdr, (uint32_t)h);
    ihdr.push_back(8); ihdr.push_back(6); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
    chunk(f, "IHDR", ihdr);
    std::vector<uint8_t> raw;
    raw.reserve((size_t)h * (4 * (size_t)w + 1));
    for (int y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgba + (size_t)y * 4 * w, rgba + (size_t)(y + 1) * 4 * w);
    }
    std::vector<uint8_t> z;
    z.push_back(0x78); z.push_back(0x01);
    size_t pos = 0;
    uint32_t a = 1, b = 0;
    for (uint8_t c : raw) {
        a = (a + c) % 65521u;
        b = (b + a) % 65521u;
    }
    do {
        size_t n = raw.size() - pos < 65535 ? raw.size() - pos : 65535;
        z.push_back(pos + n == raw.size() ? 1 : 0);
        z.push_back(n & 0xff); z.push_back(n >> 8);
        z.push_back(~n & 0xff); z.push_back((~n >> 8) & 0xff);
        z.insert(z.end(), raw.begin() + (ptrdiff_t)pos, raw.begin() + (ptrdiff_t)(pos + n));
        pos += n;
    } while (pos < raw.size());
    be32(z, (b << 16) | a);
    chunk(f, "IDAT", z);
    chunk(f, "IEND", {});
    bool ok = fclose(f) == 0;
    if (!ok) {
        rt_set_error("write failed: %s", path);
        return RT_E_IO;
    }
    return RT_OK;
}

} // namespace rt_host

// self-test hook: rt_div_by (the traversal's division) against IEEE '/' on
// random operands in and around its guarded range; returns mismatches
extern "C" unsigned long long rt_selftest_division(unsigned long long n, unsigned long long seed,
                                                   unsigned long long *tested)
{
    unsigned long long x = seed * 2654435761ull + 88172645463325252ull, bad = 0, t = 0;
    auto rnd = [&]() {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return (uint32_t)(x >> 11);
    };
    auto bits = [](uint32_t u) {
        float f;
        memcpy(&f, &u, 4);
        return f;
    };
    for (unsigned long long i = 0; i < n; ++i) {
        const uint32_t ua = rnd(), ub = rnd();
        float a, b;
        switch (i & 3) {
        case 0: a = bits(ua); b = bits(ub); break;                                  // any bits
        case 1: a = (float)(int32_t)ua * 1e-7f; b = (float)(int32_t)ub * 4.7e-10f; break; // scene-like
        case 2: // exponents inside the guard window
            a = bits((ua & 0x807fffffu) | (((ua >> 23) % 100 + 67) << 23));
            b = bits((ub & 0x807fffffu) | (((ub >> 23) % 100 + 67) << 23));
            break;
        default: // powers of two and near-guard exponents
            a = bits((ua & 0x80000000u) | (((ua >> 23) % 110 + 60) << 23) | (ua & 1u ? 0u : (ua & 0x7fffffu)));
            b = bits((ub & 0x80000000u) | (((ub >> 23) % 110 + 60) << 23) | (ub & 1u ? 0u : (ub & 0x7fffffu)));
        }
        if (!(b == b) || !(a == a)) continue;
        const float q = a / b, r = rt_div_by(a, b, rt_recip_guard(b));
        uint32_t uq, ur;
        memcpy(&uq, &q, 4);
        memcpy(&ur, &r, 4);
        ++t;
        if (uq != ur && !(q == 0.0f && r == 0.0f)) ++bad; // the sign of a zero t is never observed
    }
    if (tested) *tested = t;
    return bad;
}
