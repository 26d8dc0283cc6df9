// png_writer.cpp — 8-bit RGB PNG encoder over zlib (replaces cv::imwrite,
// raytracer/src/main.cpp:86-89) and toByte packing (core.h:313-316, main.cpp:19-34).
//
// The deflate stream can be produced by several threads: each thread
// compresses a band of filtered scanlines as an independent raw-deflate
// segment ending on a byte boundary (Z_SYNC_FLUSH, last one Z_FINISH), the
// segments are concatenated behind one zlib header and the Adler-32 values are
// merged with adler32_combine — the pigz construction.  Decoders see one
// ordinary zlib stream.
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rt.h"

namespace {

void put_u32(std::vector<unsigned char>& v, uint32_t x) {
    v.push_back((unsigned char)(x >> 24));
    v.push_back((unsigned char)(x >> 16));
    v.push_back((unsigned char)(x >> 8));
    v.push_back((unsigned char)x);
}

void put_chunk(std::vector<unsigned char>& out, const char* type, const unsigned char* data, size_t n) {
    put_u32(out, (uint32_t)n);
    size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    if (n) out.insert(out.end(), data, data + n);
    uLong crc = crc32(0L, Z_NULL, 0);
    crc = crc32(crc, out.data() + start, (uInt)(n + 4));
    put_u32(out, (uint32_t)crc);
}

// Compress one band of rows (filter byte 0 + RGB payload per row).
bool deflate_band(const uint8_t* rgb, int W, int y0, int y1, bool last, std::vector<unsigned char>& out,
                  uLong& adler, size_t& raw_len) {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, 1, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    const size_t row = (size_t)W * 3;
    std::vector<unsigned char> line(row + 1);
    out.clear();
    adler = adler32(0L, Z_NULL, 0);
    raw_len = 0;
    std::vector<unsigned char> buf(1 << 16);
    for (int y = y0; y < y1; ++y) {
        line[0] = 0;  // filter: None
        std::memcpy(line.data() + 1, rgb + (size_t)y * row, row);
        adler = adler32(adler, line.data(), (uInt)line.size());
        raw_len += line.size();
        zs.next_in = line.data();
        zs.avail_in = (uInt)line.size();
        const int flush = (y + 1 == y1) ? (last ? Z_FINISH : Z_SYNC_FLUSH) : Z_NO_FLUSH;
        do {
            zs.next_out = buf.data();
            zs.avail_out = (uInt)buf.size();
            int rc = deflate(&zs, flush);
            if (rc == Z_STREAM_ERROR) { deflateEnd(&zs); return false; }
            out.insert(out.end(), buf.data(), buf.data() + (buf.size() - zs.avail_out));
        } while (zs.avail_out == 0 || (flush != Z_NO_FLUSH && zs.avail_in > 0));
    }
    if (y0 == y1 && last) {  // empty final band: still terminate the stream
        zs.next_in = nullptr;
        zs.avail_in = 0;
        zs.next_out = buf.data();
        zs.avail_out = (uInt)buf.size();
        deflate(&zs, Z_FINISH);
        out.insert(out.end(), buf.data(), buf.data() + (buf.size() - zs.avail_out));
    }
    deflateEnd(&zs);
    return true;
}

}  // namespace

extern "C" void rt_framebuffer_to_rgb8(const double* fb, size_t n_pixels, uint8_t* rgb8) {
    for (size_t i = 0; i < n_pixels * 3; ++i) {
        double v = fb[i];
        // clamp01 (core.h:313): max(0, min(1, v)); toByte: (int)std::round(v*255)
        double c = std::min(1.0, v);
        c = std::max(0.0, c);
        rgb8[i] = (uint8_t)(int)std::round(c * 255.0);
    }
}

extern "C" int rt_write_png(const char* path, const uint8_t* rgb8, int W, int H, int n_threads) {
    if (!path || !rgb8 || W <= 0 || H <= 0) return RT_ERR_INVALID_ARG;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > H) n_threads = H;
    // Split rows into bands, compress concurrently.
    std::vector<std::vector<unsigned char>> seg(n_threads);
    std::vector<uLong> adl(n_threads);
    std::vector<size_t> lens(n_threads);
    std::vector<char> ok(n_threads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) {
        int y0 = (int)((long long)H * t / n_threads), y1 = (int)((long long)H * (t + 1) / n_threads);
        auto job = [&, t, y0, y1]() {
            ok[t] = deflate_band(rgb8, W, y0, y1, t + 1 == n_threads, seg[t], adl[t], lens[t]);
        };
        if (n_threads == 1) job(); else th.emplace_back(job);
    }
    for (auto& x : th) x.join();
    for (int t = 0; t < n_threads; ++t)
        if (!ok[t]) return RT_ERR_IO;

    std::vector<unsigned char> idat;
    idat.push_back(0x78);   // zlib header: deflate, 32K window
    idat.push_back(0x01);   // FCHECK so that (0x78<<8 | 0x01) % 31 == 0, level "fastest"
    uLong adler = adl[0];
    for (int t = 0; t < n_threads; ++t) {
        idat.insert(idat.end(), seg[t].begin(), seg[t].end());
        if (t > 0) adler = adler32_combine(adler, adl[t], (z_off_t)lens[t]);
    }
    put_u32(idat, (uint32_t)adler);

    std::vector<unsigned char> png = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    unsigned char ihdr[13];
    ihdr[0] = (unsigned char)(W >> 24); ihdr[1] = (unsigned char)(W >> 16);
    ihdr[2] = (unsigned char)(W >> 8);  ihdr[3] = (unsigned char)W;
    ihdr[4] = (unsigned char)(H >> 24); ihdr[5] = (unsigned char)(H >> 16);
    ihdr[6] = (unsigned char)(H >> 8);  ihdr[7] = (unsigned char)H;
    ihdr[8] = 8;   // bit depth
    ihdr[9] = 2;   // colour type RGB
    ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    put_chunk(png, "IHDR", ihdr, 13);
    put_chunk(png, "IDAT", idat.data(), idat.size());
    put_chunk(png, "IEND", nullptr, 0);

    FILE* f = std::fopen(path, "wb");
    if (!f) return RT_ERR_IO;
    size_t w = std::fwrite(png.data(), 1, png.size(), f);
    int rc = std::fclose(f);
    if (w != png.size() || rc != 0) return RT_ERR_IO;
    return RT_OK;
}
