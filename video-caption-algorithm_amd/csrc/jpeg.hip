// JPEG frame decode in front of the encoder: the reference's `Image.open(path).convert("RGB")`
// (core/preprocessing/frame_loader.py:42-44, libjpeg-turbo under Pillow) for baseline sequential
// Huffman JPEGs, with the same arithmetic as that decoder:
//   host  : marker parsing and entropy decoding (T.81 F.2.2; the one stage that is serial per
//           image) into quantised DCT coefficients, images decoded on parallel host threads;
//   device: dequantisation + jpeg_idct_islow (jidctint.c: 13-bit fixed-point LL&M, PASS1_BITS 2,
//           the post-IDCT range-limit table) one 8x8 block per 8 lanes, then one kernel that
//           upsamples chroma with jdsample.c's fancy (triangle) filters and converts YCbCr to RGB
//           with jdcolor.c's 16-bit fixed-point tables, writing the uint8 [n, H, W, 3] frames that
//           vcap_frames_preprocess resizes and normalises.
// Supported: 8-bit, 1 or 3 components in one interleaved scan, 4:4:4 / 4:2:2 / 4:2:0, restart
// markers.  Progressive / arithmetic / 12-bit / CMYK images are refused (VCAP_E_UNSUPPORTED).
// Parity: tests/test_gpu_jpeg.py (bit-exact against Pillow and against oracle/jpeg_oracle.py).
#include "../../include/vcap.h"
#include "vcap_common.h"
#include "vcap_kernels.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct HuffTable {
  bool present = false;
  uint16_t lut[512];  // 9-bit lookahead: (code length << 8) | symbol, 0 = longer code
  int maxcode[18], valptr[17], mincode[17];
  uint8_t vals[256];
};

struct Parsed {
  JpegInfo info;
  uint16_t qt[4][64];  // natural order
  bool qt_present[4] = {false, false, false, false};
  HuffTable dc[4], ac[4];
  int td[3], ta[3], tq[3];
  int restart = 0;
  bool jfif = false, adobe = false;  // APP0 JFIF / APP14 Adobe seen (libjpeg's colour-space guess)
  int adobe_transform = 0;
  const uint8_t* scan = nullptr;
  size_t scan_len = 0;
};

bool build_huff(HuffTable& t, const uint8_t* counts, const uint8_t* syms, int nsym) {
  std::memset(t.lut, 0, sizeof(t.lut));
  int code = 0, k = 0;
  for (int len = 1; len <= 16; ++len) {
    t.valptr[len] = k;
    t.mincode[len] = code;
    code += counts[len - 1];
    k += counts[len - 1];
    t.maxcode[len] = counts[len - 1] ? code - 1 : -1;
    if (code > (1 << len)) return false;
    code <<= 1;
  }
  t.maxcode[17] = 0x7fffffff;
  if (k != nsym) return false;
  std::memcpy(t.vals, syms, nsym);
  for (int len = 1; len <= 9; ++len)
    for (int i = 0; i < counts[len - 1]; ++i) {
      const int c = t.mincode[len] + i, s = syms[t.valptr[len] + i];
      const int lo = c << (9 - len), n = 1 << (9 - len);
      for (int j = 0; j < n; ++j) t.lut[lo + j] = (uint16_t)((len << 8) | s);
    }
  t.present = true;
  return true;
}

int parse(const uint8_t* d, size_t len, Parsed& p, std::string& err) {
  auto bad = [&](const char* m) -> int {
    err = m;
    return VCAP_E_UNSUPPORTED;
  };
  if (len < 4 || d[0] != 0xFF || d[1] != 0xD8) {
    err = "not a JPEG (no SOI)";
    return VCAP_E_ARG;
  }
  size_t i = 2;
  bool have_sof = false;
  while (i + 4 <= len) {
    if (d[i] != 0xFF) {
      err = "corrupt JPEG: marker expected";
      return VCAP_E_ARG;
    }
    while (i < len && d[i] == 0xFF) ++i;
    if (i >= len) break;
    const int m = d[i++];
    if (m == 0xD9) break;
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (i + 2 > len) break;
    const size_t seg_len = ((size_t)d[i] << 8) | d[i + 1];
    if (seg_len < 2 || i + seg_len > len) {
      err = "corrupt JPEG: segment length";
      return VCAP_E_ARG;
    }
    const uint8_t* s = d + i + 2;
    const size_t sl = seg_len - 2;
    if (m == 0xDB) {  // DQT
      size_t q = 0;
      while (q < sl) {
        const int pq = s[q] >> 4, tq = s[q] & 15;
        if (tq > 3) return bad("DQT table id");
        const size_t n = pq ? 128 : 64;
        if (q + 1 + n > sl) return bad("DQT length");
        for (int k = 0; k < 64; ++k)
          p.qt[tq][kZigzag[k]] = pq ? (uint16_t)((s[q + 1 + 2 * k] << 8) | s[q + 2 + 2 * k]) : s[q + 1 + k];
        p.qt_present[tq] = true;
        q += 1 + n;
      }
    } else if (m == 0xC0 || m == 0xC1) {  // baseline / extended sequential Huffman
      if (sl < 6 || s[0] != 8) return bad("only 8-bit JPEG samples");
      JpegInfo& f = p.info;
      f.height = (s[1] << 8) | s[2];
      f.width = (s[3] << 8) | s[4];
      f.ncomp = s[5];
      if (f.ncomp != 1 && f.ncomp != 3) return bad("1 or 3 components only");
      if (have_sof) return bad("more than one frame header");
      if (sl < 6 + 3 * (size_t)f.ncomp || f.width <= 0 || f.height <= 0) return bad("SOF length");
      if ((long)f.width * f.height > (64L << 20)) return bad("image larger than 64 Mpixel");
      f.hmax = f.vmax = 1;
      for (int k = 0; k < f.ncomp; ++k) {
        f.id[k] = s[6 + 3 * k];
        f.h[k] = s[7 + 3 * k] >> 4;
        f.v[k] = s[7 + 3 * k] & 15;
        p.tq[k] = s[8 + 3 * k];
        if (f.h[k] < 1 || f.h[k] > 2 || f.v[k] < 1 || f.v[k] > 2 || p.tq[k] > 3) return bad("sampling factors");
        f.hmax = std::max(f.hmax, f.h[k]);
        f.vmax = std::max(f.vmax, f.v[k]);
      }
      // one component = a non-interleaved scan (T.81 A.2.2): its MCU is one 8x8 block in raster
      // order over ceil(W/8) x ceil(H/8), whatever sampling factors the SOF declares (libjpeg
      // likewise walks a lone component's blocks with unit factors)
      if (f.ncomp == 1) f.h[0] = f.v[0] = f.hmax = f.vmax = 1;
      have_sof = true;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return bad("progressive / lossless / arithmetic JPEG");
    } else if (m == 0xC4) {  // DHT
      size_t q = 0;
      while (q + 17 <= sl) {
        const int tc = s[q] >> 4, th = s[q] & 15;
        int nsym = 0;
        for (int k = 0; k < 16; ++k) nsym += s[q + 1 + k];
        if (tc > 1 || th > 3 || nsym > 256 || q + 17 + nsym > sl) return bad("DHT table");
        if (!build_huff(tc ? p.ac[th] : p.dc[th], s + q + 1, s + q + 17, nsym)) return bad("DHT codes");
        q += 17 + nsym;
      }
    } else if (m == 0xDD) {  // DRI
      if (sl < 2) return bad("DRI length");
      p.restart = (s[0] << 8) | s[1];
    } else if (m == 0xE0 && sl >= 5 && std::memcmp(s, "JFIF", 5) == 0) {  // APP0 JFIF
      p.jfif = true;
    } else if (m == 0xEE && sl >= 12 && std::memcmp(s, "Adobe", 5) == 0) {  // APP14 Adobe (any position)
      p.adobe = true;
      p.adobe_transform = s[11];
    } else if (m == 0xDA) {  // SOS
      if (!have_sof) return bad("SOS before SOF");
      // colour space as libjpeg decides it (jdapimin.c default_decompress_parms) once every marker
      // before the scan is known: JFIF -> YCbCr; else Adobe transform 0 -> RGB; else component ids
      // 'R','G','B' -> RGB; else YCbCr.  Only YCbCr (or greyscale) is decoded here.
      if (p.info.ncomp == 3 && !p.jfif) {
        const bool rgb = p.adobe ? p.adobe_transform == 0
                                 : (p.info.id[0] == 'R' && p.info.id[1] == 'G' && p.info.id[2] == 'B');
        if (rgb) return bad("RGB-coded JPEG (no YCbCr transform)");
      }
      const int ns = s[0];
      if (ns != p.info.ncomp) return bad("only single-scan interleaved JPEGs");
      for (int k = 0; k < ns; ++k) {
        const int cid = s[1 + 2 * k], t = s[2 + 2 * k];
        int c = -1;
        for (int j = 0; j < p.info.ncomp; ++j)
          if (p.info.id[j] == cid) c = j;
        if (c < 0) return bad("SOS component id");
        p.td[c] = t >> 4;
        p.ta[c] = t & 15;
        if (p.td[c] > 3 || p.ta[c] > 3 || !p.dc[p.td[c]].present || !p.ac[p.ta[c]].present) return bad("SOS tables");
      }
      size_t j = i + seg_len, e = j;
      while (e + 1 < len) {
        if (d[e] == 0xFF && d[e + 1] != 0x00 && !(d[e + 1] >= 0xD0 && d[e + 1] <= 0xD7) && d[e + 1] != 0xFF) break;
        ++e;
      }
      p.scan = d + j;
      p.scan_len = e - j;
      for (int k = 0; k < p.info.ncomp; ++k)
        if (!p.qt_present[p.tq[k]]) return bad("missing quantisation table");
      JpegInfo& f = p.info;
      const int mx = (f.width + 8 * f.hmax - 1) / (8 * f.hmax), my = (f.height + 8 * f.vmax - 1) / (8 * f.vmax);
      for (int k = 0; k < f.ncomp; ++k) {
        f.bx[k] = mx * f.h[k];
        f.by[k] = my * f.v[k];
        // chroma up-sampling this decoder implements: none, h2v1 or h2v2 fancy (dw > 2, as libjpeg)
        const int fh = f.hmax / f.h[k], fv = f.vmax / f.v[k];
        const int dw = (f.width * f.h[k] + f.hmax - 1) / f.hmax;
        if (f.hmax % f.h[k] || f.vmax % f.v[k] || (fh == 1 && fv == 2) || (fh > 1 && dw <= 2))
          return bad("chroma sampling other than 4:4:4 / 4:2:2 / 4:2:0");
      }
      if (f.h[0] != f.hmax || f.v[0] != f.vmax) return bad("luma must carry the largest sampling factors");
      return 0;
    }
    i += seg_len;
  }
  err = "no scan in JPEG";
  return VCAP_E_ARG;
}

struct BitReader {
  const uint8_t *p, *end;
  uint64_t buf = 0;
  int nbits = 0;
  void fill() {
    while (nbits <= 56) {
      uint32_t b = 0;
      if (p < end) {
        b = *p;
        if (b == 0xFF) {
          if (p + 1 < end && p[1] == 0x00) {
            p += 2;
          } else {
            b = 0;  // a marker: zeros from here on, as libjpeg inserts
          }
        } else {
          ++p;
        }
      }
      buf |= (uint64_t)b << (56 - nbits);
      nbits += 8;
    }
  }
  uint32_t peek(int n) const { return (uint32_t)(buf >> (64 - n)); }
  void skip(int n) {
    buf <<= n;
    nbits -= n;
  }
  int sym(const HuffTable& t) {
    fill();
    const uint16_t e = t.lut[peek(9)];
    if (e >> 8) {
      skip(e >> 8);
      return e & 0xFF;
    }
    for (int len = 10; len <= 16; ++len) {
      const int code = (int)peek(len);
      if (code <= t.maxcode[len]) {
        skip(len);
        return t.vals[t.valptr[len] + code - t.mincode[len]];
      }
    }
    skip(16);
    return 0;  // corrupt code: libjpeg warns and continues with zeros
  }
  int receive_extend(int s) {
    if (s <= 0 || s > 16) return 0;  // (a corrupt DC table can name > 16 bits: zeros, as libjpeg warns)
    fill();
    const int v = (int)peek(s);
    skip(s);
    return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
  }
  void restart() {  // drop the padding bits, step over the RSTn marker
    buf = 0;
    nbits = 0;
    while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
    if (p + 1 < end) p += 2;
  }
};

// entropy decode one image into the component-major coefficient buffer (natural order)
void decode_coefficients(const Parsed& p, int img, int n, int16_t* coef, const size_t* comp_off) {
  const JpegInfo& f = p.info;
  const int mx = f.bx[0] / f.h[0], my = f.by[0] / f.v[0];
  BitReader br{p.scan, p.scan + p.scan_len};
  int pred[3] = {0, 0, 0};
  int16_t* base[3];
  for (int k = 0; k < f.ncomp; ++k) base[k] = coef + comp_off[k] + (size_t)img * f.bx[k] * f.by[k] * 64;
  (void)n;
  for (int mcu = 0; mcu < mx * my; ++mcu) {
    if (p.restart && mcu && mcu % p.restart == 0) {
      br.restart();
      pred[0] = pred[1] = pred[2] = 0;
    }
    const int mby = mcu / mx, mbx = mcu - mby * mx;
    for (int k = 0; k < f.ncomp; ++k) {
      const HuffTable& dct = p.dc[p.td[k]];
      const HuffTable& act = p.ac[p.ta[k]];
      for (int v = 0; v < f.v[k]; ++v)
        for (int h = 0; h < f.h[k]; ++h) {
          int16_t* blk = base[k] + ((size_t)(mby * f.v[k] + v) * f.bx[k] + (mbx * f.h[k] + h)) * 64;
          std::memset(blk, 0, 64 * sizeof(int16_t));
          const int s = br.sym(dct);
          pred[k] += br.receive_extend(s);
          blk[0] = (int16_t)pred[k];
          for (int z = 1; z < 64;) {
            const int rs = br.sym(act);
            const int r = rs >> 4, sz = rs & 15;
            if (sz == 0) {
              if (r != 15) break;
              z += 16;
              continue;
            }
            z += r;
            const int val = br.receive_extend(sz);
            if (z < 64) blk[kZigzag[z]] = (int16_t)val;
            ++z;
          }
        }
    }
  }
}

// jidctint.c constants (CONST_BITS 13, PASS1_BITS 2)
constexpr int CB = 13, P1 = 2;
constexpr int F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633;
constexpr int F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

std::mutex g_stage_mu;
void* g_stage = nullptr;  // pinned host staging of the coefficients (process lifetime)
size_t g_stage_bytes = 0;

}  // namespace

// ---------------------------------------------------------------------------------------------
// jidctint.c jpeg_idct_islow, one 8x8 block per 8 lanes: lane c runs the column pass of column c
// (dequantising), then the row pass of row c (through LDS).  JLONG arithmetic as 64-bit long.
__device__ __forceinline__ void vcap_idct_1d(const long (&d)[8], long (&r)[8]) {
  long z2 = d[2], z3 = d[6];
  long z1 = (z2 + z3) * F0541;
  const long tmp2 = z1 + z3 * (-F1847), tmp3 = z1 + z2 * F0765;
  const long tmp0 = (d[0] + d[4]) * (1L << CB), tmp1 = (d[0] - d[4]) * (1L << CB);
  const long tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  long t0 = d[7], t1 = d[5], t2 = d[3], t3 = d[1];
  z1 = t0 + t3;
  z2 = t1 + t2;
  z3 = t0 + t2;
  long z4 = t1 + t3;
  const long z5 = (z3 + z4) * F1175;
  t0 *= F0298;
  t1 *= F2053;
  t2 *= F3072;
  t3 *= F1501;
  z1 *= -F0899;
  z2 *= -F2562;
  z3 = z3 * (-F1961) + z5;
  z4 = z4 * (-F0390) + z5;
  t0 += z1 + z3;
  t1 += z2 + z4;
  t2 += z2 + z3;
  t3 += z1 + z4;
  r[0] = tmp10 + t3;
  r[7] = tmp10 - t3;
  r[1] = tmp11 + t2;
  r[6] = tmp11 - t2;
  r[2] = tmp12 + t1;
  r[5] = tmp12 - t1;
  r[3] = tmp13 + t0;
  r[4] = tmp13 - t0;
}

// post-IDCT range_limit[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table)
__device__ __forceinline__ uint32_t vcap_jpeg_range(long v) {
  const int y = (int)(v & 1023);
  return y < 128 ? (uint32_t)(y + 128) : y < 512 ? 255u : y < 896 ? 0u : (uint32_t)(y - 896);
}

// qt: this component's table of image 0; image i's is qt + i * qt_stride (frames of one clip may
// carry different tables: ffmpeg's MJPEG rate control writes a per-frame qscale into each DQT).
__global__ __launch_bounds__(256) void vcap_jpeg_idct_kernel(const int16_t* __restrict__ coef,
                                                             const uint16_t* __restrict__ qt, int qt_stride,
                                                             uint8_t* __restrict__ plane, int bx, int by,
                                                             long nblocks) {
  __shared__ int ws[32][8][9];  // [block][row][col] (+1 pad)
  const int t = threadIdx.x, lb = t >> 3, c = t & 7;
  const long blk0 = (long)blockIdx.x * 32 + lb;
  const bool live = blk0 < nblocks;
  const long blk = live ? blk0 : 0;
  const long per_img = (long)bx * by;
  const long img = blk / per_img, rem = blk - img * per_img;
  const int16_t* in = coef + blk * 64;
  qt += img * qt_stride;
  // pass 1: column c, dequantised (the all-AC-zero shortcut is the same arithmetic)
  long d[8], r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = (long)in[k * 8 + c] * qt[k * 8 + c];
  vcap_idct_1d(d, r);
#pragma unroll
  for (int k = 0; k < 8; ++k) ws[lb][k][c] = (int)((r[k] + (1L << (CB - P1 - 1))) >> (CB - P1));
  __syncthreads();
  // pass 2: row c
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = ws[lb][c][k];
  vcap_idct_1d(d, r);
  if (!live) return;
  uint32_t px[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) px[k] = vcap_jpeg_range((r[k] + (1L << (CB + P1 + 3 - 1))) >> (CB + P1 + 3));
  const int byi = (int)(rem / bx), bxi = (int)(rem - (long)byi * bx);
  uint8_t* o = plane + img * per_img * 64 + ((long)(byi * 8 + c) * bx * 8) + bxi * 8;
  *reinterpret_cast<u32x2*>(o) =
      (u32x2){px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24), px[4] | (px[5] << 8) | (px[6] << 16) | (px[7] << 24)};
}

struct JpegPlanes {
  const uint8_t* p[3];
  int stride[3];     // padded plane width (bx * 8)
  int plane_sz[3];   // bytes per image per plane
  int dw[3], dh[3];  // downsampled (real) width / height
  int fh[3], fv[3];  // upsampling factors
};

// jdsample.c fancy upsampling of one chroma sample at output (x, y)
__device__ __forceinline__ int vcap_jpeg_chroma(const uint8_t* pl, int stride, int dw, int dh, int fh, int fv, int x,
                                                int y) {
  if (fh == 1) return pl[(long)y * stride + x];
  const int ix = x >> 1, u = x & 1;
  if (fv == 1) {  // h2v1_fancy_upsample
    const uint8_t* row = pl + (long)y * stride;
    const int c = row[ix];
    if (u == 0) return ix == 0 ? c : (3 * c + row[ix - 1] + 1) >> 2;
    return ix == dw - 1 ? c : (3 * c + row[ix + 1] + 2) >> 2;
  }
  // h2v2_fancy_upsample: column sums of the nearest and next-nearest input rows (image top /
  // bottom rows replicated as the context rows)
  const int iy = y >> 1;
  const int ny = (y & 1) ? min(iy + 1, dh - 1) : max(iy - 1, 0);
  const uint8_t* r0 = pl + (long)iy * stride;
  const uint8_t* r1 = pl + (long)ny * stride;
  auto cs = [&](int k) { return 3 * (int)r0[k] + (int)r1[k]; };
  const int th = cs(ix);
  if (u == 0) return ix == 0 ? (th * 4 + 8) >> 4 : (th * 3 + cs(ix - 1) + 8) >> 4;
  return ix == dw - 1 ? (th * 4 + 7) >> 4 : (th * 3 + cs(ix + 1) + 7) >> 4;
}

__global__ __launch_bounds__(256) void vcap_jpeg_color_kernel(JpegPlanes pl, int ncomp, int W, int H, long total,
                                                              uint8_t* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const long img = i / ((long)W * H);
  const int rem = (int)(i - img * W * H), y = rem / W, x = rem - y * W;
  const int yv = pl.p[0][img * pl.plane_sz[0] + (long)y * pl.stride[0] + x];
  uint8_t* o = out + i * 3;
  if (ncomp == 1) {
    o[0] = o[1] = o[2] = (uint8_t)yv;
    return;
  }
  const int cb = vcap_jpeg_chroma(pl.p[1] + img * pl.plane_sz[1], pl.stride[1], pl.dw[1], pl.dh[1], pl.fh[1], pl.fv[1], x, y);
  const int cr = vcap_jpeg_chroma(pl.p[2] + img * pl.plane_sz[2], pl.stride[2], pl.dw[2], pl.dh[2], pl.fh[2], pl.fv[2], x, y);
  // jdcolor.c build_ycc_rgb_table: FIX(x) = x * 2^16 + 0.5, ONE_HALF = 2^15
  const int xcb = cb - 128, xcr = cr - 128;
  const int crr = (91881 * xcr + 32768) >> 16;
  const int cbb = (116130 * xcb + 32768) >> 16;
  const int gof = (-22554 * xcb + 32768 + -46802 * xcr) >> 16;
  o[0] = (uint8_t)min(max(yv + crr, 0), 255);
  o[1] = (uint8_t)min(max(yv + gof, 0), 255);
  o[2] = (uint8_t)min(max(yv + cbb, 0), 255);
}

// ---------------------------------------------------------------------------------------------
int vcap_jpeg_header(const uint8_t* data, size_t len, JpegInfo* info, std::string* err) {
  Parsed p;
  std::string e;
  const int rc = parse(data, len, p, e);
  if (rc) {
    if (err) *err = e;
    return rc;
  }
  *info = p.info;
  return 0;
}

static void jpeg_layout(const JpegInfo& f, int n, size_t* comp_off, size_t* coef_elems, size_t* plane_off,
                        size_t* plane_bytes) {
  size_t co = 0, po = 0;
  for (int k = 0; k < f.ncomp; ++k) {
    comp_off[k] = co;
    co += (size_t)n * f.bx[k] * f.by[k] * 64;
    plane_off[k] = po;
    po += ((size_t)n * f.bx[k] * f.by[k] * 64 + 255) & ~(size_t)255;
  }
  *coef_elems = co;
  *plane_bytes = po;
}

size_t vcap_jpeg_ws_bytes(const JpegInfo& f, int n) {
  size_t co[3], ce, po[3], pb;
  jpeg_layout(f, n, co, &ce, po, &pb);
  return ((ce * sizeof(int16_t) + 255) & ~(size_t)255) + pb + (size_t)n * 3 * 64 * sizeof(uint16_t) + 256;
}

int vcap_jpeg_decode(const uint8_t* const* data, const size_t* lens, int n, uint8_t* out, void* ws, size_t ws_bytes,
                     hipStream_t s, std::string* err) {
  std::vector<Parsed> ps(n);
  std::string e;
  for (int i = 0; i < n; ++i) {
    const int rc = parse(data[i], lens[i], ps[i], e);
    if (rc) {
      *err = "image " + std::to_string(i) + ": " + e;
      return rc;
    }
    const JpegInfo &a = ps[0].info, &b = ps[i].info;
    bool same = a.width == b.width && a.height == b.height && a.ncomp == b.ncomp;
    for (int k = 0; same && k < a.ncomp; ++k) same = a.h[k] == b.h[k] && a.v[k] == b.v[k];
    if (!same) {
      *err = "image " + std::to_string(i) + ": size or chroma sampling differs from image 0";
      return VCAP_E_UNSUPPORTED;
    }
  }
  const JpegInfo& f = ps[0].info;
  if ((long)n * f.width * f.height > (1L << 31) / 3) {
    *err = "batch larger than 2 GiB of RGB";
    return VCAP_E_UNSUPPORTED;
  }
  if (ws_bytes < vcap_jpeg_ws_bytes(f, n)) {
    *err = "workspace too small";
    return VCAP_E_WORKSPACE;
  }
  size_t comp_off[3], coef_elems, plane_off[3], plane_bytes;
  jpeg_layout(f, n, comp_off, &coef_elems, plane_off, &plane_bytes);
  // entropy decode: the serial stage, one host thread per group of images, into a pinned staging
  // buffer (kept for the process: pageable memory halved the upload rate of the coefficients,
  // which are n x 128 B per 8x8 block)
  std::lock_guard<std::mutex> lock(g_stage_mu);
  const size_t stage_need = ((coef_elems * sizeof(int16_t) + 15) & ~(size_t)15) + (size_t)n * 3 * 64 * sizeof(uint16_t);
  if (g_stage_bytes < stage_need) {
    if (g_stage) (void)hipHostFree(g_stage);
    g_stage = nullptr;
    g_stage_bytes = 0;
    const size_t want = stage_need + stage_need / 4;
    if (hipHostMalloc(&g_stage, want, hipHostMallocDefault) != hipSuccess) {
      g_stage = nullptr;
      *err = "jpeg decode: pinned staging allocation failed";
      return -(int)hipErrorOutOfMemory;
    }
    g_stage_bytes = want;
  }
  int16_t* coef = (int16_t*)g_stage;
  const int nt = std::max(1, std::min<int>({n, (int)std::thread::hardware_concurrency(), 16}));
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (int i = next++; i < n; i = next++) decode_coefficients(ps[i], i, n, coef, comp_off);
    });
  for (auto& t : th) t.join();
  char* w = (char*)ws;
  int16_t* d_coef = (int16_t*)w;
  uint8_t* d_planes = (uint8_t*)(w + ((coef_elems * sizeof(int16_t) + 255) & ~(size_t)255));
  uint16_t* d_qt = (uint16_t*)(d_planes + plane_bytes);
  // every image's own tables, [image][component][64] natural order, staged behind the coefficients
  uint16_t* qts = (uint16_t*)((char*)g_stage + ((coef_elems * sizeof(int16_t) + 15) & ~(size_t)15));
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < f.ncomp; ++k) std::memcpy(qts + ((size_t)i * f.ncomp + k) * 64, ps[i].qt[ps[i].tq[k]], 128);
  hipError_t he = hipMemcpyAsync(d_coef, coef, coef_elems * sizeof(int16_t), hipMemcpyHostToDevice, s);
  // from here on the pinned staging buffer may be read by an in-flight copy: every return below
  // synchronises the stream first (the next call reuses or frees the buffer)
  const bool enqueued = he == hipSuccess;
  if (he == hipSuccess)
    he = hipMemcpyAsync(d_qt, qts, sizeof(uint16_t) * 64 * f.ncomp * (size_t)n, hipMemcpyHostToDevice, s);
  for (int k = 0; k < f.ncomp && he == hipSuccess; ++k) {
    const long nb = (long)n * f.bx[k] * f.by[k];
    hipLaunchKernelGGL(vcap_jpeg_idct_kernel, dim3((unsigned)((nb + 31) / 32)), dim3(256), 0, s, d_coef + comp_off[k],
                       d_qt + 64 * k, 64 * f.ncomp, d_planes + plane_off[k], f.bx[k], f.by[k], nb);
    he = hipGetLastError();
  }
  if (he == hipSuccess) {
    JpegPlanes pl{};
    for (int k = 0; k < f.ncomp; ++k) {
      pl.p[k] = d_planes + plane_off[k];
      pl.stride[k] = f.bx[k] * 8;
      pl.plane_sz[k] = f.bx[k] * f.by[k] * 64;
      pl.fh[k] = f.hmax / f.h[k];
      pl.fv[k] = f.vmax / f.v[k];
      pl.dw[k] = (f.width * f.h[k] + f.hmax - 1) / f.hmax;
      pl.dh[k] = (f.height * f.v[k] + f.vmax - 1) / f.vmax;
    }
    const long total = (long)n * f.width * f.height;
    hipLaunchKernelGGL(vcap_jpeg_color_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, pl, f.ncomp,
                       f.width, f.height, total, out);
    he = hipGetLastError();
  }
  // the staging buffer is reused by the next call: the copies must have finished, on every path
  if (enqueued) {
    const hipError_t hs = hipStreamSynchronize(s);
    if (he == hipSuccess) he = hs;
  }
  if (he != hipSuccess) {
    *err = std::string("jpeg decode: ") + hipGetErrorString(he);
    return -(int)he;
  }
  return 0;
}
