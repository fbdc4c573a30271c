// sgpu_seq.cpp -- headless sequence stacking: the host side of Siril's
// scripting path `stack <seq> ...` (command.c:11985 process_stackone ->
// stack_one_seq :11729 -> main_stack stacking.c:76 -> stack_mean_or_median
// median_and_mean.c:1261) for regular FITS, FITSEQ and SER sequences, mono
// or three-layer (RGB).
//
//   * .seq reader: io/seqfile.c:84-500 -- S (quoted or bare name, beg,
//     number, selnum, fixed, reference, version, ...), T (TS = SER, the .ser
//     next to the .seq; TF = FITSEQ, <name>.fit[s]), L, I (filenum, incl) and
//     R<layer> registration lines (v4+: `fwhm wfwhm round quality bkg nstars
//     H h00..h22`; v1-3: shiftx shifty first); the registration layer is the
//     first layer with data (get_registration_layer, registration.c:34-47) and
//     an invalid reference image is replaced by sequence_find_refimage's
//     choice (io/sequence.c:1791-1846);
//   * frames: regular sequences read seqname + %0{fixed}d + extension
//     (io/sequence.c:1335-1352); FITSEQ: every image HDU of one file
//     (io/fits_sequence.c:39-120); SER: frame i of the .ser file
//     (io/ser.c:257-382, 1054-1213: 178-byte header, 8- or 16-bit samples
//     with the inverted endianness flag, RGB/BGR interleaved planes, top-down
//     rows, timestamp trailer);
//   * FITS: BITPIX -32 (float; Siril's [0, 1] rescale of ADU-valued floats),
//     16 (BZERO 32768 or signed, DATA_USHORT) or 8 (DATA_USHORT), NAXIS3 1 or 3,
//     big-endian, 2880-byte blocks;
//   * block reader: stack_read_block_data (median_and_mean.c:382-545) in FITS
//     row order -- output row R reads input row R - shifty with zero fill
//     (Siril reads top-down areas -- FITS partial reads flipped, SER rows as
//     stored -- and writes row H-1-y: the net map on FITS-order rows is the
//     identity shifted by the registration dy = -h12, SER row t being
//     FITS-order row H-1-t); the x shift round_to_int(h02) is applied on the
//     device (median_and_mean.c:1615-1636);
//   * compute: sgpu_stack_rows / sgpu_stack_rows_u16 per block and layer, the
//     next block read by a second thread while the GPU stacks the current one;
//   * result: BITPIX -32 (float input or use_32bit_output) or 16 with BZERO
//     32768, saved like savefits (command.c:11772); -rejmap / -rejmaps files
//     (command.c:11592-11602, 11778-11803): counts * (1.0f / N) as float
//     images named <out>_low+high_rejmap / _low_rejmap / _high_rejmap.
// Normalization (params->normalize != NO_NORM with no coefficient arrays):
// compute_normalization (stacking/normalization.c:249-294) -- each included
// frame is read whole (unshifted) per layer, its estimators computed on the
// GPU (norm_stats.hip, STATS_NORM or STATS_LITENORM) and turned into
// coefficients relative to the reference image (sgpu_norm_factors).
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdlib>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sgpu_internal.h"
#include "sirilgpu.h"

using sgpu_host::fail;

namespace {

// ------------------------------------------------------------------ images
// One frame of a sequence: a FITS HDU (regular sequence or FITSEQ) or a SER
// frame.  `bitpix` is the engine's sample type: -32 float, 16 WORD (8-bit
// data are widened to WORD, as Siril reads them into DATA_USHORT).
enum Kind { K_FITS = 0, K_SER = 1 };
struct Img {
    int kind = K_FITS;
    std::string path;
    long w = 0, h = 0;
    int nlayers = 1;
    int bitpix = 0;               // -32 or 16
    long long data_off = 0;       // byte offset of the frame's samples
    // FITS
    int file_bitpix = 0;          // -32, 16, 8
    double bzero = 0.0, bscale = 1.0;
    bool has_datamax = false;     // DATAMAX card present
    double datamax = 0.0;
    bool from_siril = false;      // PROGRAM card contains "Siril" (io/fits_keywords.c:1281)
    unsigned stackcnt = 1;        // STACKCNT, else NCOMBINE (image_format_fits.c:62,1086-1095); 1 if absent
    bool has_stackcnt = false;
    // SER
    int ser_depth = 2;            // bytes per sample
    int ser_big_endian = 0;       // the header flag as Siril reads it (SER_BIG_ENDIAN = 1, ser.h)
    int ser_color = 0;            // SER_MONO 0, SER_RGB 100, SER_BGR 101 (Bayer ids read as mono)
};

// How float data of a FITS file is brought to Siril's [0, 1] range.
enum ReadMode {
    READ_RAW = 0,      // stored values (format helpers)
    READ_PARTIAL = 1,  // internal_read_partial_fits (image_format_fits.c:994-1007): the block reader
    READ_WHOLE = 2     // readfits -> read_fits_with_convert (:861-910): whole frames (normalization)
};

double card_num(const char *card) {
    const char *eq = std::strchr(card, '=');
    if (!eq || eq - card > 9) return NAN;
    return std::strtod(eq + 1, nullptr);
}

std::string card_str(const char *card) {
    const char *q0 = (const char *)std::memchr(card + 10, '\'', 70);
    const char *q1 = q0 ? (const char *)std::memchr(q0 + 1, '\'', card + 80 - q0 - 1) : nullptr;
    return (q0 && q1) ? std::string(q0 + 1, q1) : std::string();
}

// Parse the header of the HDU at byte `off`.  Returns 0 and fills `f` (is_image
// when the HDU holds a >= 2-D image) and `next` (offset of the following HDU);
// 1 at end of file.
int parse_hdu(FILE *fp, long long off, Img &f, bool &is_image, long long &next, std::string &extname) {
    if (std::fseek(fp, (long)off, SEEK_SET) != 0) return 1;
    char block[2880];
    long naxis = -1, n[3] = {0, 0, 1};
    bool end = false, xtension_image = (off == 0);
    long nblocks = 0;
    int bitpix = 0;
    extname.clear();
    while (!end) {
        if (std::fread(block, 1, 2880, fp) != 2880) return nblocks == 0 ? 1 : -1;
        nblocks++;
        for (int c = 0; c < 36 && !end; c++) {
            const char *card = block + 80 * c;
            char key[9];
            std::memcpy(key, card, 8);
            key[8] = 0;
            for (int i = 7; i >= 0 && key[i] == ' '; i--) key[i] = 0;
            if (!std::strcmp(key, "END")) end = true;
            else if (!std::strcmp(key, "XTENSION")) xtension_image = card_str(card).rfind("IMAGE", 0) == 0;
            else if (!std::strcmp(key, "BITPIX")) bitpix = (int)card_num(card);
            else if (!std::strcmp(key, "NAXIS")) naxis = (long)card_num(card);
            else if (!std::strcmp(key, "NAXIS1")) n[0] = (long)card_num(card);
            else if (!std::strcmp(key, "NAXIS2")) n[1] = (long)card_num(card);
            else if (!std::strcmp(key, "NAXIS3")) n[2] = (long)card_num(card);
            else if (!std::strcmp(key, "BZERO")) f.bzero = card_num(card);
            else if (!std::strcmp(key, "BSCALE")) f.bscale = card_num(card);
            else if (!std::strcmp(key, "EXTNAME")) extname = card_str(card);
            else if (!std::strcmp(key, "DATAMAX")) {
                const double v = card_num(card);
                if (v == v) {
                    f.has_datamax = true;
                    f.datamax = v;
                }
            } else if (!std::strcmp(key, "PROGRAM")) {
                f.from_siril = card_str(card).find("Siril") != std::string::npos;
            } else if (!std::strcmp(key, "STACKCNT") || (!std::strcmp(key, "NCOMBINE") && !f.has_stackcnt)) {
                // __tryToFindKeywords: STACKCNT first, NCOMBINE otherwise (TUINT)
                const double v = card_num(card);
                if (v == v && v >= 0) {
                    f.stackcnt = (unsigned)v;
                    f.has_stackcnt = !std::strcmp(key, "STACKCNT");
                }
            }
        }
    }
    long long nbytes = naxis > 0 ? (long long)std::abs(bitpix) / 8 : 0;
    for (int a = 0; a < naxis && a < 3; a++) nbytes *= n[a];
    f.kind = K_FITS;
    f.file_bitpix = bitpix;
    f.w = n[0];
    f.h = n[1];
    f.nlayers = (int)n[2];
    f.data_off = off + nblocks * 2880LL;
    next = f.data_off + (nbytes + 2879) / 2880 * 2880;
    is_image = xtension_image && naxis >= 2 && n[0] > 0 && n[1] > 0;
    return 0;
}

int check_fits_type(Img &f) {
    if (f.nlayers != 1 && f.nlayers != 3)
        return fail(SGPU_SEQUENCE_ERROR, "FITS images must have 1 or 3 planes");
    if (f.file_bitpix == -32) {
        // physical BZERO/BSCALE float scaling (image_format_fits.c:988-993) is not supported
        if (f.bzero != 0.0 || f.bscale != 1.0)
            return fail(SGPU_SEQUENCE_ERROR, "scaled float FITS (BZERO/BSCALE) is not supported");
        f.bitpix = -32;
    } else if (f.file_bitpix == 16) {
        // unsigned convention (BZERO 32768) and plain signed shorts both read
        // as DATA_USHORT stored + 32768 (src/tests/fits_scaling_test.c:190-205,
        // :317-332); physical float scaling of 16-bit data is not supported
        if (f.bscale != 1.0 || (f.bzero != 32768.0 && f.bzero != 0.0))
            return fail(SGPU_SEQUENCE_ERROR, "scaled 16-bit FITS (BSCALE/BZERO) is not supported");
        f.bitpix = 16;
    } else if (f.file_bitpix == 8) {
        if (f.bscale != 1.0 || f.bzero != 0.0)
            return fail(SGPU_SEQUENCE_ERROR, "scaled 8-bit FITS (BSCALE/BZERO) is not supported");
        f.bitpix = 16;                    // BYTE_IMG data live in WORD buffers (DATA_USHORT)
    } else {
        return fail(SGPU_SEQUENCE_ERROR, "FITS BITPIX must be -32, 16 or 8");
    }
    return SGPU_OK;
}

// the primary image of a FITS file (or the first image extension)
int fits_open(const char *path, Img &f) {
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return fail(SGPU_SEQUENCE_ERROR, (std::string("cannot open FITS ") + path).c_str());
    long long off = 0, next = 0;
    int rc = 1;
    std::string ext;
    for (;;) {
        Img g;
        g.path = path;
        bool img = false;
        const int e = parse_hdu(fp, off, g, img, next, ext);
        if (e) {
            rc = fail(SGPU_SEQUENCE_ERROR, e < 0 ? std::string("no END card in ") + path
                                                 : std::string("no 2-D image in ") + path);
            break;
        }
        if (img) {
            f = g;
            rc = check_fits_type(f);
            break;
        }
        off = next;
    }
    std::fclose(fp);
    return rc;
}

// every image HDU of a FITS sequence file (fits_sequence.c:39-120: image HDUs
// with NAXIS > 1, skipping ICC / thumbnail / HST auxiliary extensions; HDUs
// whose size or type differs from the first one are skipped)
int fitseq_open(const char *path, std::vector<Img> &frames) {
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return fail(SGPU_SEQUENCE_ERROR, (std::string("cannot open FITSEQ ") + path).c_str());
    frames.clear();
    long long off = 0, next = 0;
    std::string ext;
    int rc = SGPU_OK;
    for (;;) {
        Img g;
        g.path = path;
        bool img = false;
        const int e = parse_hdu(fp, off, g, img, next, ext);
        if (e > 0) break;
        if (e < 0) {
            rc = fail(SGPU_SEQUENCE_ERROR, std::string("truncated FITS sequence ") + path);
            break;
        }
        off = next;
        if (!img) continue;
        bool skip = false;
        for (const char *pfx : {"ICCProfile", "Thumbnail", "HDRLET", "WCS", "D2IM"})
            skip = skip || ext.rfind(pfx, 0) == 0;
        if (skip) continue;
        if (check_fits_type(g)) {
            rc = SGPU_SEQUENCE_ERROR;
            break;
        }
        if (!frames.empty() && (g.w != frames[0].w || g.h != frames[0].h || g.nlayers != frames[0].nlayers ||
                                g.file_bitpix != frames[0].file_bitpix))
            continue;
        frames.push_back(g);
    }
    std::fclose(fp);
    if (!rc && frames.size() < 2) rc = fail(SGPU_SEQUENCE_ERROR, "a FITS sequence needs at least 2 images");
    return rc;
}

// ------------------------------------------------------------------- SER
struct SerInfo {
    std::string file_id;
    int lu_id = 0, color_id = 0, endian = 0, w = 0, h = 0, bit_depth = 0;
    unsigned frame_count = 0;
    char observer[40] = {0}, instrument[40] = {0}, telescope[40] = {0};
    uint64_t date = 0, date_utc = 0;
    std::vector<uint64_t> ts;
    int depth_bytes = 2, planes = 1;
};

inline uint32_t le32(const unsigned char *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline uint64_t le64(const unsigned char *p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

// ser_read_header + ser_read_timestamp (io/ser.c:106-178, 257-382)
int ser_open(const char *path, SerInfo &s, std::vector<Img> *frames) {
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return fail(SGPU_SEQUENCE_ERROR, (std::string("cannot open SER ") + path).c_str());
    unsigned char hd[178];
    std::fseek(fp, 0, SEEK_END);
    const long long fsize = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    if (std::fread(hd, 1, 178, fp) != 178) {
        std::fclose(fp);
        return fail(SGPU_SEQUENCE_ERROR, std::string("short SER header in ") + path);
    }
    s = SerInfo();
    s.file_id.assign((const char *)hd, 14);
    s.lu_id = (int)le32(hd + 14);
    s.color_id = (int)le32(hd + 18);
    s.endian = (int)le32(hd + 22);
    s.w = (int)le32(hd + 26);
    s.h = (int)le32(hd + 30);
    s.bit_depth = (int)le32(hd + 34);
    s.frame_count = le32(hd + 38);
    std::memcpy(s.observer, hd + 42, 40);
    std::memcpy(s.instrument, hd + 82, 40);
    std::memcpy(s.telescope, hd + 122, 40);
    s.observer[39] = s.instrument[39] = s.telescope[39] = 0;
    s.date = le64(hd + 162);
    s.date_utc = le64(hd + 170);
    const bool bayer = s.color_id >= 8 && s.color_id <= 11;
    if (s.color_id != 0 && !bayer && s.color_id != 100 && s.color_id != 101) {
        std::fclose(fp);
        return fail(SGPU_SEQUENCE_ERROR, "Cannot handle this SER type (" + std::to_string(s.color_id) + ")");
    }
    if (s.w <= 0 || s.h <= 0 || s.bit_depth <= 0 || s.bit_depth > 16) {
        std::fclose(fp);
        return fail(SGPU_SEQUENCE_ERROR, "Invalid SER header dimensions");
    }
    s.depth_bytes = s.bit_depth <= 8 ? 1 : 2;
    s.planes = (s.color_id == 100 || s.color_id == 101) ? 3 : 1;
    const long long fbytes = (long long)s.w * s.h * s.planes * s.depth_bytes;
    if (s.frame_count == 0)   // ser_recompute_frame_count (:179-200)
        s.frame_count = (unsigned)((fsize - 178) / fbytes);
    const long long ts_off = 178 + fbytes * s.frame_count;
    if (fsize >= ts_off + 8LL * s.frame_count) {
        s.ts.resize(s.frame_count);
        std::vector<unsigned char> t(8ull * s.frame_count);
        std::fseek(fp, (long)ts_off, SEEK_SET);
        if (std::fread(t.data(), 1, t.size(), fp) == t.size())
            for (unsigned i = 0; i < s.frame_count; i++) s.ts[i] = le64(&t[8ull * i]);
        else
            s.ts.clear();
    }
    std::fclose(fp);
    if (fsize < 178 + fbytes * (long long)s.frame_count)
        return fail(SGPU_SEQUENCE_ERROR, std::string("truncated SER file ") + path);
    if (frames) {
        frames->clear();
        for (unsigned i = 0; i < s.frame_count; i++) {
            Img g;
            g.kind = K_SER;
            g.path = path;
            g.w = s.w;
            g.h = s.h;
            g.nlayers = s.planes;
            g.bitpix = 16;
            g.data_off = 178 + fbytes * (long long)i;
            g.ser_depth = s.depth_bytes;
            g.ser_big_endian = s.endian;
            g.ser_color = bayer ? 0 : s.color_id;   // CFA read as monochrome (no open_debayer)
            frames->push_back(g);
        }
    }
    return SGPU_OK;
}

inline uint32_t be32(const unsigned char *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// max over all samples of a float file, in float (fit_stats, image_format_fits.c:84-140)
int fits_float_max(const Img &f, float &mx);

// convert_floats (image_format_fits.c:648-672) for FLOAT_IMG: falls through to
// the USHORT case, data[i] * INV_USHRT_MAX_SINGLE in float
inline void convert_floats(float *d, size_t n) {
    for (size_t i = 0; i < n; i++) d[i] = d[i] * 0.000015259022f;   // INV_USHRT_MAX_SINGLE
}

// rows [r0, r0+n) of layer `layer` in FITS row order into dst (float or WORD
// per element, row-major, width w); rows outside [0, h) are zero-filled.
// Float files are brought to [0, 1] like Siril reads them (mode):
//  READ_PARTIAL: DATAMAX card, or when absent the max of the 3 (or 4)
//    samples dest[0], dest[n/3], ... of the region actually read (the rows
//    inside the image), `> 10` -> convert_floats (image_format_fits.c:994-1007);
//  READ_WHOLE: keywords.data_max, which is the file's true max for files not
//    written by Siril (fits_keywords.c:1281-1288) and DATAMAX (or 0) otherwise,
//    `> 10` -> convert_floats (:906-910).
// SER frames: file rows are top-down, FITS-order row q is SER row h-1-q
// (ser_read_opened_partial reads areas top-down and the stack writes row
// H-1-y); 8-bit samples are widened, 16-bit ones byte-swapped per the header
// flag (ser_manage_endianess_and_depth, ser.c:521-539); RGB/BGR planes are
// de-interleaved (crop_area_from_color_lines, ser.c:1027-1044).
int read_rows(const Img &f, int layer, long r0, long n, void *dst, std::vector<unsigned char> &tmp,
              int mode = READ_RAW) {
    const int es = f.bitpix == -32 ? 4 : 2;
    std::memset(dst, 0, (size_t)n * f.w * es);
    const long a = std::max(r0, 0L), b = std::min(r0 + n, f.h);
    if (a >= b) return SGPU_OK;
    FILE *fp = std::fopen(f.path.c_str(), "rb");
    if (!fp) return fail(SGPU_SEQUENCE_ERROR, (std::string("cannot open ") + f.path).c_str());
    const size_t cnt = (size_t)(b - a) * f.w;
    if (f.kind == K_SER) {
        const size_t rowb = (size_t)f.w * f.nlayers * f.ser_depth;
        const long s0 = f.h - b;   // SER rows [h-b, h-a)
        tmp.resize((size_t)(b - a) * rowb);
        if (std::fseek(fp, (long)(f.data_off + (long long)s0 * rowb), SEEK_SET) != 0 ||
            std::fread(tmp.data(), 1, tmp.size(), fp) != tmp.size()) {
            std::fclose(fp);
            return fail(SGPU_SEQUENCE_ERROR, (std::string("short read in ") + f.path).c_str());
        }
        std::fclose(fp);
        const int coff = f.nlayers == 3 ? (f.ser_color == 101 ? 2 - layer : layer) : 0;
        uint16_t *o = (uint16_t *)dst + (size_t)(a - r0) * f.w;
        for (long q = a; q < b; q++) {
            const unsigned char *row = tmp.data() + (size_t)((f.h - 1 - q) - s0) * rowb;
            uint16_t *orow = o + (size_t)(q - a) * f.w;
            for (long x = 0; x < f.w; x++) {
                const size_t e = (size_t)x * f.nlayers + coff;
                if (f.ser_depth == 1) {
                    orow[x] = row[e];
                } else {
                    const unsigned char *pp = row + 2 * e;
                    orow[x] = f.ser_big_endian == 1 ? (uint16_t)((pp[0] << 8) | pp[1]) : (uint16_t)(pp[0] | (pp[1] << 8));
                }
            }
        }
        return SGPU_OK;
    }
    const int fes = std::abs(f.file_bitpix) / 8;
    const size_t bytes = cnt * fes;
    tmp.resize(bytes);
    const long long plane = (long long)f.w * f.h * fes * layer;
    if (std::fseek(fp, (long)(f.data_off + plane + (long long)a * f.w * fes), SEEK_SET) != 0 ||
        std::fread(tmp.data(), 1, bytes, fp) != bytes) {
        std::fclose(fp);
        return fail(SGPU_SEQUENCE_ERROR, (std::string("short read in ") + f.path).c_str());
    }
    std::fclose(fp);
    if (f.file_bitpix == -32) {
        uint32_t *o = (uint32_t *)dst + (size_t)(a - r0) * f.w;
        for (size_t i = 0; i < cnt; i++) o[i] = be32(&tmp[4 * i]);
        float *d = (float *)o;
        bool rescale = false;
        if (mode == READ_PARTIAL) {
            if (f.has_datamax) {
                rescale = f.datamax > 10.0;
            } else if (cnt > 3) {
                double dm = 0.0;   // data_max = max(data_max, dest[i]) from 0
                for (size_t i = 0; i < cnt; i += cnt / 3) dm = std::max(dm, (double)d[i]);
                rescale = dm > 10.0;
            }
        } else if (mode == READ_WHOLE) {
            double dm = f.has_datamax ? f.datamax : 0.0;
            if (!f.from_siril) {
                float mx;
                if (int r = fits_float_max(f, mx)) return r;
                dm = (double)mx;
            }
            rescale = dm > 10.0;
        }
        if (rescale) convert_floats(d, cnt);
    } else if (f.file_bitpix == 16) {
        uint16_t *o = (uint16_t *)dst + (size_t)(a - r0) * f.w;
        for (size_t i = 0; i < cnt; i++)   // signed big-endian + BZERO 32768
            o[i] = (uint16_t)((((uint16_t)tmp[2 * i] << 8) | tmp[2 * i + 1]) ^ 0x8000u);
    } else {
        uint16_t *o = (uint16_t *)dst + (size_t)(a - r0) * f.w;
        for (size_t i = 0; i < cnt; i++) o[i] = tmp[i];
    }
    return SGPU_OK;
}

int fits_float_max(const Img &f, float &mx) {
    mx = -1.E33f;
    std::vector<unsigned char> tmp;
    const long step = std::max(1L, (64L << 20) / (f.w * 4));
    std::vector<float> chunk;
    for (int l = 0; l < f.nlayers; l++) {
        for (long r = 0; r < f.h; r += step) {
            const long nr = std::min(step, f.h - r);
            chunk.resize((size_t)nr * f.w);
            if (int e = read_rows(f, l, r, nr, chunk.data(), tmp, READ_RAW)) return e;
            for (float v : chunk) mx = (v > mx) ? v : mx;
        }
    }
    return SGPU_OK;
}

void put_card(std::string &hdr, const char *key, const std::string &val, const char *comment = nullptr) {
    char c[81];
    if (comment)
        std::snprintf(c, sizeof c, "%-8.8s= %20s / %-47.47s", key, val.c_str(), comment);
    else
        std::snprintf(c, sizeof c, "%-8.8s= %20s%50s", key, val.c_str(), "");
    hdr.append(c, 80);
}

// FITS header of an image HDU (SIMPLE ... END, padded to 2880 bytes)
std::string fits_header(long w, long h, int nlayers, int bitpix, const std::vector<std::string> &history) {
    std::string hdr;
    put_card(hdr, "SIMPLE", "T", "conforms to FITS standard");
    put_card(hdr, "BITPIX", std::to_string(bitpix), "array data type");
    put_card(hdr, "NAXIS", nlayers > 1 ? "3" : "2", "number of array dimensions");
    put_card(hdr, "NAXIS1", std::to_string(w));
    put_card(hdr, "NAXIS2", std::to_string(h));
    if (nlayers > 1) put_card(hdr, "NAXIS3", std::to_string(nlayers));
    if (bitpix == 16) {
        put_card(hdr, "BZERO", "32768", "offset data range to that of unsigned short");
        put_card(hdr, "BSCALE", "1", "default scaling factor");
    }
    for (const std::string &s : history) {
        char c[81];
        std::snprintf(c, sizeof c, "HISTORY %-72.72s", s.c_str());
        hdr.append(c, 80);
    }
    char end[81];
    std::snprintf(end, sizeof end, "%-80s", "END");
    hdr.append(end, 80);
    hdr.append((2880 - hdr.size() % 2880) % 2880, ' ');
    return hdr;
}

int fits_es(int bitpix) { return bitpix == -32 ? 4 : bitpix == 8 ? 1 : 2; }

// samples [a, b) of `data` (float for BITPIX -32, WORD otherwise) in FITS
// big-endian form at dst[0 ..)
void fits_convert(const void *data, size_t a, size_t b, int es, unsigned char *dst) {
    if (es == 4) {
        const uint32_t *in = (const uint32_t *)data;
        for (size_t i = a; i < b; i++) {
            const uint32_t v = __builtin_bswap32(in[i]);
            std::memcpy(dst + 4 * (i - a), &v, 4);
        }
    } else if (es == 2) {
        const uint16_t *in = (const uint16_t *)data;
        for (size_t i = a; i < b; i++) {
            const uint16_t v = __builtin_bswap16((uint16_t)(in[i] ^ 0x8000u));
            std::memcpy(dst + 2 * (i - a), &v, 2);
        }
    } else {                      // BYTE_IMG from WORD samples (whole numbers <= 255 here)
        const uint16_t *in = (const uint16_t *)data;
        for (size_t i = a; i < b; i++) dst[i - a] = (unsigned char)(in[i] > 255 ? 255 : in[i]);
    }
}

int fits_write(const char *path, const void *data, long w, long h, int nlayers, int bitpix,
               const std::vector<std::string> &history) {
    const std::string hdr = fits_header(w, h, nlayers, bitpix, history);
    const int es = fits_es(bitpix);
    const size_t cnt = (size_t)w * h * nlayers;
    const size_t pad = (2880 - (cnt * es) % 2880) % 2880;
    // the file image (header, big-endian samples, padding), converted by a
    // few threads: a 6000 x 4000 float result is 96 MB
    std::vector<unsigned char> img(hdr.size() + cnt * es + pad, 0);
    std::memcpy(img.data(), hdr.data(), hdr.size());
    unsigned char *dst = img.data() + hdr.size();
    const int nt = (int)std::max<size_t>(1, std::min<size_t>(8, cnt >> 20));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) {
        const size_t a = cnt * t / nt, b = cnt * (t + 1) / nt;
        pool.emplace_back(fits_convert, data, a, b, es, dst + a * es);
    }
    fits_convert(data, 0, cnt / nt, es, dst);
    for (std::thread &th : pool) th.join();
    FILE *fp = std::fopen(path, "wb");
    if (!fp) return fail(SGPU_GENERIC_ERROR, (std::string("cannot write ") + path).c_str());
    bool ok = std::fwrite(img.data(), 1, img.size(), fp) == img.size();
    ok = (std::fclose(fp) == 0) && ok;
    return ok ? SGPU_OK : fail(SGPU_GENERIC_ERROR, (std::string("write failed: ") + path).c_str());
}

// The result image written while the stack runs: the header and the file's
// size first, then each block's rows (converted to FITS order) by a writer
// thread as soon as they are back on the host, under the next block's copy
// and stack.  Used unless -output_norm needs the whole image first.  The rows
// go to a temporary file next to the result, renamed over it only after the
// last write and close succeeded: a stack that fails part-way leaves no
// partial image and keeps any earlier result at that path (the temporary is
// unlinked on every error path, including the destructor's).
struct FitsStream {
    int fd = -1;
    size_t hdr = 0;
    int es = 4;
    std::thread th;
    int err = 0;
    std::string tmp, dst;
    int open(const char *path, long w, long h, int nlayers, int bitpix, const std::vector<std::string> &history) {
        const std::string hs = fits_header(w, h, nlayers, bitpix, history);
        es = fits_es(bitpix);
        hdr = hs.size();
        const size_t cnt = (size_t)w * h * nlayers;
        const size_t total = hdr + cnt * es + (2880 - (cnt * es) % 2880) % 2880;
        dst = path;
        tmp = dst + ".sgpu-part";
        fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0) return fail(SGPU_GENERIC_ERROR, (std::string("cannot write ") + tmp).c_str());
        if (::pwrite(fd, hs.data(), hdr, 0) != (ssize_t)hdr || ::ftruncate(fd, (off_t)total) != 0) {
            discard();
            return fail(SGPU_GENERIC_ERROR, (std::string("write failed: ") + path).c_str());
        }
        return SGPU_OK;
    }
    // samples [o, o + n) of data; the previous block's write is joined first
    void emit(const void *data, size_t o, size_t n) {
        join();
        th = std::thread([this, data, o, n] {
            std::vector<unsigned char> buf(n * es);
            fits_convert(data, o, o + n, es, buf.data());
            size_t done = 0;
            while (done < buf.size()) {
                const ssize_t w = ::pwrite(fd, buf.data() + done, buf.size() - done, (off_t)(hdr + o * es + done));
                if (w <= 0) {
                    err = 1;
                    return;
                }
                done += (size_t)w;
            }
        });
    }
    void join() {
        if (th.joinable()) th.join();
    }
    // the result is complete: close, then move the temporary over the path
    int close() {
        join();
        const int c = fd >= 0 ? ::close(fd) : 0;
        fd = -1;
        if (err || c != 0) {
            discard();
            return fail(SGPU_GENERIC_ERROR, "writing the result failed");
        }
        if (::rename(tmp.c_str(), dst.c_str()) != 0) {
            discard();
            return fail(SGPU_GENERIC_ERROR, (std::string("cannot rename the result to ") + dst).c_str());
        }
        tmp.clear();
        return SGPU_OK;
    }
    // an unfinished result: close and remove the temporary
    void discard() {
        join();
        if (fd >= 0) ::close(fd);
        fd = -1;
        if (!tmp.empty()) ::unlink(tmp.c_str());
        tmp.clear();
    }
    ~FitsStream() { discard(); }
};

// ------------------------------------------------------------------- .seq
struct Seq {
    std::string dir, name, path;
    int beg = 0, number = 0, selnum = 0, fixed = 0, reference = 0, version = -1;
    char type = 0;                    // 0 regular, 'S' SER, 'F' FITSEQ
    int nb_layers = 1;
    std::vector<int> filenum, incl;
    static constexpr int kLayers = 10;
    std::vector<double> dx[kLayers], dy[kLayers];
    // regdata (core/siril.h) with the reference's types: fwhm, weighted_fwhm,
    // roundness, background_lvl float; quality double; number_of_stars int
    std::vector<float> fwhm[kLayers], wfwhm[kLayers], roundness[kLayers], bkg[kLayers];
    std::vector<double> quality[kLayers];
    std::vector<int> nstars[kLayers];
    bool has_reg[kLayers] = {false};
};

int round_to_int(double x) {        // core/proto.h:208-213
    x = std::min(x, 2147483647.0 - 0.5);
    x = std::max(x, -2147483648.0 + 0.5);
    return (int)(x + (x >= 0.0 ? 0.5 : -0.5));
}

int read_seq(const char *path, Seq &q) {
    std::string p(path);
    if (p.size() < 4 || p.compare(p.size() - 4, 4, ".seq") != 0) p += ".seq";
    FILE *fp = std::fopen(p.c_str(), "r");
    if (!fp) return fail(SGPU_SEQUENCE_ERROR, ("cannot open sequence " + p).c_str());
    const size_t slash = p.find_last_of('/');
    q = Seq();
    q.path = p;
    q.dir = slash == std::string::npos ? "" : p.substr(0, slash + 1);
    char line[512];
    int ni = 0, nr[Seq::kLayers] = {0};
    bool have_s = false;
    int err = SGPU_OK;
    while (std::fgets(line, sizeof line, fp)) {
        if (line[0] == 'S' && line[1] == ' ') {
            char name[512] = {0};
            int var = 0, fz = 0, dz = 0;
            const char *fmt = (line[2] == '\'') ? "'%511[^']' %d %d %d %d %d %d %d %d %d"
                                                : "%511s %d %d %d %d %d %d %d %d %d";
            const int nt = std::sscanf(line + 2, fmt, name, &q.beg, &q.number, &q.selnum, &q.fixed,
                                       &q.reference, &q.version, &var, &fz, &dz);
            if (nt < 6 || q.number < 1) { err = fail(SGPU_SEQUENCE_ERROR, "bad S line"); break; }
            if (var || fz || dz) { err = fail(SGPU_SEQUENCE_ERROR, "variable/fz/drizzle sequences not supported"); break; }
            q.name = name;
            q.filenum.assign(q.number, 0);
            q.incl.assign(q.number, 0);
            for (int l = 0; l < Seq::kLayers; l++) {
                q.dx[l].assign(q.number, 0.0);
                q.dy[l].assign(q.number, 0.0);
                q.fwhm[l].assign(q.number, 0.f);
                q.wfwhm[l].assign(q.number, 0.f);
                q.roundness[l].assign(q.number, 0.f);
                q.bkg[l].assign(q.number, 0.f);
                q.quality[l].assign(q.number, 0.0);
                q.nstars[l].assign(q.number, 0);
            }
            have_s = true;
        } else if (line[0] == 'T') {
            if (line[1] == 'S' || line[1] == 'F') {
                q.type = line[1];
            } else {
                err = fail(SGPU_SEQUENCE_ERROR, "unsupported sequence type (T line)");
                break;
            }
        } else if (line[0] == 'L' && line[1] == ' ') {
            if (std::sscanf(line + 2, "%d", &q.nb_layers) != 1) { err = fail(SGPU_SEQUENCE_ERROR, "bad L line"); break; }
        } else if (line[0] == 'I' && line[1] == ' ') {
            if (!have_s || ni >= q.number) { err = fail(SGPU_SEQUENCE_ERROR, "bad I line"); break; }
            if (std::sscanf(line + 2, "%d %d", &q.filenum[ni], &q.incl[ni]) != 2) {
                err = fail(SGPU_SEQUENCE_ERROR, "bad I line");
                break;
            }
            ni++;
        } else if (line[0] == 'R' && line[1] >= '0' && line[1] <= '9') {
            const int l = line[1] - '0';
            if (!have_s || nr[l] >= q.number) { err = fail(SGPU_SEQUENCE_ERROR, "bad R line"); break; }
            const int k = nr[l];
            // io/seqfile.c:352-421, one format per .seq version
            float sx = 0.f, sy = 0.f;
            if (q.version >= 4) {
                double H[9];
                if (std::sscanf(line + 3, "%g %g %g %lg %g %d H %lg %lg %lg %lg %lg %lg %lg %lg %lg", &q.fwhm[l][k],
                                &q.wfwhm[l][k], &q.roundness[l][k], &q.quality[l][k], &q.bkg[l][k], &q.nstars[l][k],
                                &H[0], &H[1], &H[2], &H[3], &H[4], &H[5], &H[6], &H[7], &H[8]) != 15) {
                    err = fail(SGPU_SEQUENCE_ERROR, "bad R line");
                    break;
                }
                q.dx[l][k] = H[2];       // translation_from_H: dx = h02, dy = -h12
                q.dy[l][k] = -H[5];
            } else {
                int ok;
                if (q.version < 1) {
                    float rcx, rcy, angle;
                    const int nt = std::sscanf(line + 3, "%f %f %g %g %g %g %lg", &sx, &sy, &rcx, &rcy, &angle,
                                               &q.fwhm[l][k], &q.quality[l][k]);
                    if (nt == 3) q.quality[l][k] = rcx;          // old format: quality third
                    ok = nt == 7 || nt == 3;
                } else if (q.version <= 2) {
                    ok = std::sscanf(line + 3, "%f %f %g %g %lg", &sx, &sy, &q.fwhm[l][k], &q.roundness[l][k],
                                     &q.quality[l][k]) == 5;
                } else {
                    ok = std::sscanf(line + 3, "%f %f %g %g %g %lg", &sx, &sy, &q.fwhm[l][k], &q.wfwhm[l][k],
                                     &q.roundness[l][k], &q.quality[l][k]) == 6;
                }
                if (!ok) { err = fail(SGPU_SEQUENCE_ERROR, "bad R line"); break; }
                q.dx[l][k] = sx;         // H_from_translation(shiftx, shifty)
                q.dy[l][k] = sy;
            }
            nr[l]++;
            q.has_reg[l] = true;
        }
    }
    std::fclose(fp);
    if (err) return err;
    if (!have_s || ni != q.number) return fail(SGPU_SEQUENCE_ERROR, "sequence file incomplete");
    return SGPU_OK;
}

// get_registration_layer in scripts (registration.c:37-46): first layer with data
int registration_layer(const Seq &q) {
    for (int l = 0; l < std::max(q.nb_layers, 1) && l < Seq::kLayers; l++)
        if (q.has_reg[l]) return l;
    return -1;
}

// sequence_find_refimage (io/sequence.c:1791-1846), restated literally
int find_refimage(const Seq &q) {
    if (q.reference != -1 && q.reference >= 0 && q.reference < q.number) return q.reference;
    int best = -1;
    for (int layer = 0; layer < std::max(q.nb_layers, 1) && layer < Seq::kLayers; layer++) {
        if (!q.has_reg[layer]) continue;
        bool use_fwhm;
        double best_val;
        if (q.fwhm[layer][0] > 0.0) {
            use_fwhm = true;
            best_val = 1000000.0;
        } else if (q.quality[layer][0] > 0.0) {
            use_fwhm = false;
            best_val = 0.0;
        } else {
            continue;
        }
        for (int image = 0; image < q.number; image++) {
            if (!q.incl[image]) continue;
            if (use_fwhm && q.fwhm[layer][image] > 0 && q.fwhm[layer][image] < best_val) {
                best_val = q.fwhm[layer][image];
                best = image;
            } else if (q.quality[layer][image] > 0 && q.quality[layer][image] > best_val) {
                best_val = q.quality[layer][image];
                best = image;
            }
        }
    }
    if (best == -1) {
        for (int image = 0; image < q.number; image++)
            if (q.incl[image]) {
                best = image;
                break;
            }
    }
    return best < 0 ? 0 : best;
}

std::string frame_path(const Seq &q, int filenum) {
    char num[32];
    std::snprintf(num, sizeof num, "%0*d", q.fixed, filenum);
    for (const char *ext : {".fit", ".fits", ".fts"}) {
        const std::string p = q.dir + q.name + num + ext;
        if (FILE *fp = std::fopen(p.c_str(), "rb")) {
            std::fclose(fp);
            return p;
        }
    }
    return q.dir + q.name + num + ".fit";
}

// the frames of a sequence, in sequence order (io/seqfile.c:426-485)
int open_frames(const Seq &q, std::vector<Img> &all) {
    all.clear();
    const std::string base = q.path.substr(0, q.path.size() - 4);
    if (q.type == 'S') {
        SerInfo si;
        if (int r = ser_open((base + ".ser").c_str(), si, &all)) return r;
    } else if (q.type == 'F') {
        int r = SGPU_SEQUENCE_ERROR;
        for (const char *ext : {".fit", ".fits", ".fts"}) {
            const std::string fn = base + ext;
            if (FILE *fp = std::fopen(fn.c_str(), "rb")) {
                std::fclose(fp);
                r = fitseq_open(fn.c_str(), all);
                break;
            }
        }
        if (r) return r == SGPU_SEQUENCE_ERROR ? fail(r, "FITS sequence file not found for " + q.path) : r;
    } else {
        return SGPU_OK;   // regular: one file per frame, opened on demand
    }
    if ((int)all.size() < q.number) return fail(SGPU_SEQUENCE_ERROR, "sequence has more images than its file");
    return SGPU_OK;
}

std::string replace_ext(const std::string &path, const std::string &new_ext) {
    const size_t slash = path.find_last_of('/');
    const size_t dot = path.find_last_of('.');
    if (dot == std::string::npos || (slash != std::string::npos && dot < slash)) return path + new_ext;
    return path.substr(0, dot) + new_ext;
}

}  // namespace

extern "C" int sgpu_fits_info(const char *path, long *width, long *height, int *bitpix) {
    if (!path) return fail(SGPU_BAD_ARGUMENT, "null path");
    Img f;
    if (int r = fits_open(path, f)) return r;
    if (width) *width = f.w;
    if (height) *height = f.h;
    if (bitpix) *bitpix = f.file_bitpix == 8 ? 16 : f.bitpix;
    return SGPU_OK;
}

extern "C" int sgpu_fits_layers(const char *path) {
    if (!path) return fail(SGPU_BAD_ARGUMENT, "null path");
    Img f;
    if (int r = fits_open(path, f)) return r;
    return f.nlayers;
}

extern "C" int sgpu_image_read_rows(const char *path, int frame, int layer, long row0, long nrows, void *out,
                                    int mode) {
    if (!path || !out || nrows < 0 || frame < 0 || layer < 0 || mode < READ_RAW || mode > READ_WHOLE)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    std::string p(path);
    std::vector<Img> all;
    if (p.size() > 4 && p.compare(p.size() - 4, 4, ".ser") == 0) {
        SerInfo si;
        if (int r = ser_open(path, si, &all)) return r;
    } else if (frame == 0) {
        Img f;
        if (int r = fits_open(path, f)) return r;
        all.push_back(f);
    } else if (int r = fitseq_open(path, all)) {
        return r;
    }
    if (frame >= (int)all.size() || layer >= all[frame].nlayers) return fail(SGPU_BAD_ARGUMENT, "no such frame/layer");
    std::vector<unsigned char> tmp;
    return read_rows(all[frame], layer, row0, nrows, out, tmp, mode);
}

extern "C" int sgpu_fits_read_rows_ex(const char *path, long row0, long nrows, void *out, int mode) {
    return sgpu_image_read_rows(path, 0, 0, row0, nrows, out, mode);
}

extern "C" int sgpu_fits_read_rows(const char *path, long row0, long nrows, void *out) {
    return sgpu_fits_read_rows_ex(path, row0, nrows, out, READ_RAW);
}

extern "C" int sgpu_fits_write(const char *path, const void *data, long width, long height, int bitpix) {
    if (!path || !data || width < 1 || height < 1 || (bitpix != -32 && bitpix != 16))
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    return fits_write(path, data, width, height, 1, bitpix, {});
}

extern "C" int sgpu_fits_write_planes(const char *path, const void *data, long width, long height, int nlayers,
                                      int bitpix) {
    if (!path || !data || width < 1 || height < 1 || (nlayers != 1 && nlayers != 3) ||
        (bitpix != -32 && bitpix != 16))
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    return fits_write(path, data, width, height, nlayers, bitpix, {});
}

// ---- SER files (fixtures and the reader's own checks) ----------------------
extern "C" int sgpu_ser_write(const char *path, const void *frames, int nframes, int width, int height,
                              int color_id, int bit_depth, int endian_flag, const int64_t *unix_seconds,
                              const char *observer, uint64_t date_utc) {
    if (!path || !frames || nframes < 1 || width < 1 || height < 1 || bit_depth < 1 || bit_depth > 16)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    const int planes = (color_id == 100 || color_id == 101) ? 3 : 1;
    const int db = bit_depth <= 8 ? 1 : 2;
    unsigned char hd[178];
    std::memset(hd, 0, sizeof hd);
    std::memcpy(hd, "LUCAM-RECORDER", 14);
    auto put32 = [&](int off, uint32_t v) { for (int i = 0; i < 4; i++) hd[off + i] = (unsigned char)(v >> (8 * i)); };
    auto put64 = [&](int off, uint64_t v) { for (int i = 0; i < 8; i++) hd[off + i] = (unsigned char)(v >> (8 * i)); };
    put32(14, 0);
    put32(18, (uint32_t)color_id);
    put32(22, (uint32_t)endian_flag);
    put32(26, (uint32_t)width);
    put32(30, (uint32_t)height);
    put32(34, (uint32_t)bit_depth);
    put32(38, (uint32_t)nframes);
    if (observer) std::strncpy((char *)hd + 42, observer, 39);
    put64(162, date_utc);
    put64(170, date_utc);
    FILE *fp = std::fopen(path, "wb");
    if (!fp) return fail(SGPU_GENERIC_ERROR, std::string("cannot write ") + path);
    bool ok = std::fwrite(hd, 1, 178, fp) == 178;
    // frames: [nframes][height][width][planes] WORD samples (top-down rows, as stored)
    const size_t n = (size_t)nframes * height * width * planes;
    std::vector<unsigned char> buf(n * db);
    const uint16_t *src = (const uint16_t *)frames;
    for (size_t i = 0; i < n; i++) {
        if (db == 1) buf[i] = (unsigned char)src[i];
        else if (endian_flag == 1) { buf[2 * i] = (unsigned char)(src[i] >> 8); buf[2 * i + 1] = (unsigned char)src[i]; }
        else { buf[2 * i] = (unsigned char)src[i]; buf[2 * i + 1] = (unsigned char)(src[i] >> 8); }
    }
    ok = ok && std::fwrite(buf.data(), 1, buf.size(), fp) == buf.size();
    if (unix_seconds) {   // date_time_to_ser_timestamp (core/siril_date.c:195-199)
        for (int i = 0; i < nframes && ok; i++) {
            const uint64_t ts = (uint64_t)(unix_seconds[i] * 10000000LL) + 621355968000000000ULL;
            unsigned char t[8];
            for (int b = 0; b < 8; b++) t[b] = (unsigned char)(ts >> (8 * b));
            ok = std::fwrite(t, 1, 8, fp) == 8;
        }
    }
    ok = (std::fclose(fp) == 0) && ok;
    return ok ? SGPU_OK : fail(SGPU_GENERIC_ERROR, std::string("write failed: ") + path);
}

extern "C" int sgpu_ser_info(const char *path, int *width, int *height, int *frame_count, int *color_id,
                             int *bit_depth, int *endian_flag, char observer[40], uint64_t *date_utc,
                             int64_t *unix_seconds, int max_ts) {
    if (!path) return fail(SGPU_BAD_ARGUMENT, "null path");
    SerInfo s;
    if (int r = ser_open(path, s, nullptr)) return r;
    if (width) *width = s.w;
    if (height) *height = s.h;
    if (frame_count) *frame_count = (int)s.frame_count;
    if (color_id) *color_id = s.color_id;
    if (bit_depth) *bit_depth = s.bit_depth;
    if (endian_flag) *endian_flag = s.endian;
    if (observer) std::memcpy(observer, s.observer, 40);
    if (date_utc) *date_utc = s.date_utc;
    int nts = 0;
    if (unix_seconds) {   // ser_timestamp_to_date_time (core/siril_date.c:173-188), whole seconds
        for (size_t i = 0; i < s.ts.size() && (int)i < max_ts; i++, nts++)
            unix_seconds[i] = (int64_t)((s.ts[i] - 621355968000000000ULL) / 10000000ULL);
    }
    return nts;
}

namespace {

// ---------------------------------------------------------- frame selection
// core/sequence_filtering.c: the predicates (:45-121; the background and star
// count filters test roundness > 0, as the reference does), the thresholds
// from a percentage or a k-sigma clip of the sequence's values (:364-452) and
// the combination (:219-302).
enum FiltKind { F_INCL, F_FWHM, F_WFWHM, F_ROUND, F_BKG, F_NBSTARS, F_QUALITY };

double reg_value(const Seq &q, int layer, int i, int kind) {
    switch (kind) {
        case F_FWHM: return q.fwhm[layer][i];
        case F_WFWHM: return q.wfwhm[layer][i];
        case F_ROUND: return q.roundness[layer][i];
        case F_BKG: return q.bkg[layer][i];
        case F_NBSTARS: return (double)q.nstars[layer][i];
        default: return q.quality[layer][i];
    }
}

bool filter_pass(const Seq &q, int layer, int i, int kind, double p) {
    if (kind == F_INCL) return q.incl[i] != 0;
    if (layer < 0) return false;
    switch (kind) {
        case F_FWHM: return q.fwhm[layer][i] > 0.0f && q.fwhm[layer][i] <= p;
        case F_WFWHM: return q.wfwhm[layer][i] > 0.0f && q.wfwhm[layer][i] <= p;
        case F_ROUND: return q.roundness[layer][i] > 0.0f && q.roundness[layer][i] >= p;
        case F_BKG: return q.roundness[layer][i] > 0.0f && q.bkg[layer][i] <= p;
        case F_NBSTARS: return q.roundness[layer][i] > 0.0f && q.nstars[layer][i] >= (int)p;
        default: return q.quality[layer][i] > 0.0 && q.quality[layer][i] >= p;
    }
}

// generic_compute_accepted_value (:366-404)
double accepted_value(const Seq &q, int layer, double percent, bool lower_is_better, int kind) {
    const double extreme = lower_is_better ? DBL_MAX : DBL_MIN;
    if (layer < 0) return 0.0;
    std::vector<double> val(q.number);
    for (int i = 0; i < q.number; i++) {
        const double d = reg_value(q, layer, i, kind);
        val[i] = d <= 0.0f ? extreme : d;
    }
    std::sort(val.begin(), val.end());
    int nwd = q.number;
    if (val[q.number - 1] == extreme) {
        int i = 0;
        while (i < q.number && val[i] != extreme) i++;
        nwd = i;
    }
    const double images_number = (double)(nwd - 1);
    if (lower_is_better) {
        const double t = val[(int)(percent * images_number / 100.0)];
        return t == extreme ? 0.0 : t;
    }
    return val[(int)((100.0 - percent) * images_number / 100.0)];
}

// generic_compute_accepted_value_with_rejection (:408-452): gsl_stats_median_
// from_sorted_data and gsl_stats_sd (GSL's running mean / variance in long
// double, variance * n / (n - 1))
double accepted_value_ksigma(const Seq &q, int layer, double k, bool lower_is_better, int kind) {
    const double factor = lower_is_better ? 1. : -1;
    if (layer < 0) return 0.0;
    std::vector<double> val;
    for (int i = 0; i < q.number; i++) {
        const double d = reg_value(q, layer, i, kind);
        if (d > 0.0f) val.push_back(d * factor);
    }
    if (val.empty()) return 0.0;
    std::sort(val.begin(), val.end());
    int n = (int)val.size(), j;
    do {
        j = 0;
        const int lhs = (n - 1) / 2, rhs = n / 2;
        const double m = lhs == rhs ? val[lhs] : (val[lhs] + val[rhs]) / 2.0;
        long double mean = 0;
        for (int i = 0; i < n; i++) mean += (val[i] - mean) / (i + 1);
        const double dmean = (double)mean;
        long double var = 0;
        for (int i = 0; i < n; i++) {
            const long double delta = (val[i] - dmean);
            var += (delta * delta - var) / (i + 1);
        }
        const double sd = std::sqrt((double)var * ((double)n / ((double)n - 1.0)));
        const double t = m + k * sd;
        for (int i = n; i > 0; i--) {
            if (val[i - 1] > t) j++;
            else break;
        }
        n -= j;
    } while (j > 0);
    if (n <= 0) return 0.0;
    return factor * val[n - 1];
}

// frames the stack uses (setup_filtered_data, :305-355); returns the error
int select_frames(const Seq &q, const sgpu_stack_seq_options &o, std::vector<int> &idx) {
    struct { float lit, pct; int k; int kind; bool lower; } fl[] = {
        {o.f_fwhm, o.f_fwhm_p, o.f_fwhm_k, F_FWHM, true}, {o.f_wfwhm, o.f_wfwhm_p, o.f_wfwhm_k, F_WFWHM, true},
        {o.f_round, o.f_round_p, o.f_round_k, F_ROUND, false}, {o.f_bkg, o.f_bkg_p, o.f_bkg_k, F_BKG, true},
        {o.f_nbstars, o.f_nbstars_p, o.f_nbstars_k, F_NBSTARS, false},
        {o.f_quality, o.f_quality_p, o.f_quality_k, F_QUALITY, false}};
    if ((o.f_fwhm_p > 0.0f && o.f_fwhm > 0.0f) || (o.f_wfwhm_p > 0.0f && o.f_wfwhm > 0.0f) ||
        (o.f_round_p > 0.0f && o.f_round > 0.0f) || (o.f_quality_p > 0.0f && o.f_quality > 0.0f))
        return fail(SGPU_BAD_ARGUMENT, "Sequence filter: values can only be either literal or percent");
    const int layer = registration_layer(q);
    std::vector<std::pair<int, double>> filters;
    if (o.filter_included) filters.push_back({F_INCL, 0.0});
    for (auto &f : fl) {
        if (f.pct > 0.0f || f.lit > 0.0f) {
            double p = f.lit;
            if (!(f.lit > 0.f))
                p = f.k ? accepted_value_ksigma(q, layer, f.pct, f.lower, f.kind)
                        : accepted_value(q, layer, f.pct, f.lower, f.kind);
            filters.push_back({f.kind, p});
        }
    }
    idx.clear();
    for (int i = 0; i < q.number; i++) {
        bool ok = true;
        for (auto &f : filters) ok = ok && filter_pass(q, layer, i, f.first, f.second);
        if (ok) idx.push_back(i);
    }
    if (idx.size() < 2)
        return fail(SGPU_GENERIC_ERROR, "Provided filtering options do not allow at least two images to be processed.");
    return SGPU_OK;
}

// compute_wfwhm_weights / compute_nbstars_weights (median_and_mean.c:1137-1230)
// for one layer (every layer gets the same values)
int frame_weights(const Seq &q, int reglayer, const std::vector<int> &idx, int kind, std::vector<double> &w) {
    const int N = (int)idx.size();
    w.assign(N, 0.0);
    if (reglayer < 0 || !q.has_reg[reglayer])
        return fail(SGPU_GENERIC_ERROR, "Sequence does not have registration info, cannot use weighing");
    double norm = 0.0;
    if (kind == SGPU_WFWHM_WEIGHT) {
        double fmin = DBL_MAX, fmax = -DBL_MAX;
        for (int i : idx) {
            const double v = q.wfwhm[reglayer][i];
            if (v < fmin && v > 0) fmin = v;
            if (v > fmax) fmax = v;
        }
        const double invdenom = 1. / (1. / (fmin * fmin) - 1. / (fmax * fmax));
        const double invfwhmax2 = 1. / (fmax * fmax);
        for (int k = 0; k < N; k++) {
            const double v = q.wfwhm[reglayer][idx[k]];
            if (v > 0) {
                w[k] = (1. / (v * v) - invfwhmax2) * invdenom;
                norm += w[k];
            }
        }
        norm /= (double)N;
        if (!norm) return fail(SGPU_GENERIC_ERROR, "wFWHM weights: null norm");
    } else {
        int smin = INT_MAX, smax = 0;
        for (int i : idx) {
            smin = std::min(smin, q.nstars[reglayer][i]);
            smax = std::max(smax, q.nstars[reglayer][i]);
        }
        const double invdenom = smax == smin ? 1.0 : 1. / (double)(smax - smin);
        for (int k = 0; k < N; k++) {
            const int s = q.nstars[reglayer][idx[k]];
            w[k] = smax == smin ? 1. : (double)(s - smin) * (double)(s - smin) * invdenom * invdenom;
            norm += w[k];
        }
        norm /= (double)N;
    }
    for (double &x : w) x /= norm;
    return SGPU_OK;
}

// maximize framing: place the frame's rows into canvas rows at column dx
// (the x shift moves from the kernel into the reader)
void place_rows(const unsigned char *src, long w_in, unsigned char *dst, long w_out, long nr, int dx, int es) {
    std::memset(dst, 0, (size_t)nr * w_out * es);
    const long x0 = std::max(0L, (long)dx), x1 = std::min(w_out, w_in + dx);
    if (x0 >= x1) return;
    for (long r = 0; r < nr; r++)
        std::memcpy(dst + ((size_t)r * w_out + x0) * es, src + ((size_t)r * w_in + (x0 - dx)) * es,
                    (size_t)(x1 - x0) * es);
}

}  // namespace

extern "C" int sgpu_stack_seq_opts(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                                   int use_registration, int use_32bit_output, const char *out_path,
                                   uint64_t counts[2], const sgpu_stack_seq_options *opts);

extern "C" int sgpu_stack_seq_ex2(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                                  int use_registration, int use_32bit_output, const char *out_path,
                                  uint64_t counts[2], long max_block_bytes, int lite_norm, int rejmaps) {
    // the pre-options entry points stack the .seq's included frames (ABI 3
    // behaviour: callers size critical values / weights / shifts for them)
    sgpu_stack_seq_options o;
    std::memset(&o, 0, sizeof o);
    o.filter_included = 1;
    o.lite_norm = lite_norm;
    o.rejmaps = rejmaps;
    o.max_block_bytes = max_block_bytes;
    return sgpu_stack_seq_opts(ctx, seq_path, params, use_registration, use_32bit_output, out_path, counts, &o);
}

extern "C" int sgpu_stack_seq_ex(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                                 int use_registration, int use_32bit_output, const char *out_path,
                                 uint64_t counts[2], long max_block_bytes, int lite_norm) {
    return sgpu_stack_seq_ex2(ctx, seq_path, params, use_registration, use_32bit_output, out_path, counts,
                              max_block_bytes, lite_norm, 0);
}

extern "C" int sgpu_stack_seq(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                              int use_registration, int use_32bit_output, const char *out_path,
                              uint64_t counts[2], long max_block_bytes) {
    return sgpu_stack_seq_ex2(ctx, seq_path, params, use_registration, use_32bit_output, out_path, counts,
                              max_block_bytes, 0, 0);
}

extern "C" int sgpu_stack_seq_frames(const char *seq_path, const sgpu_stack_seq_options *opts, int *indices,
                                     int cap, int *nframes, int *ref_image) {
    if (!seq_path || !opts || !nframes) return fail(SGPU_BAD_ARGUMENT, "null argument");
    Seq q;
    if (int r = read_seq(seq_path, q)) return r;
    std::vector<int> idx;
    if (int r = select_frames(q, *opts, idx)) return r;
    *nframes = (int)idx.size();
    for (int k = 0; k < (int)idx.size() && k < cap && indices; k++) indices[k] = idx[k];
    if (ref_image) {
        const int refi = find_refimage(q);
        *ref_image = std::find(idx.begin(), idx.end(), refi) != idx.end() ? refi : idx[0];
    }
    return SGPU_OK;
}

// Siril's row-block plan (stack_compute_parallel_blocks and
// refine_blocks_candidate, stacking/median_and_mean.c:255-356).  It decides
// which rows a feather mask is upscaled over (stack_read_block_data :483-525),
// so a -feather= stack reproduces it; the result is otherwise block-free.
namespace {
int ceil_multiple(int x, int factor) {   // round_to_ceiling_multiple (core/proto.h:295-299)
    const int r = x % factor;
    return x + (factor - r) * (r != 0);
}
int refine_candidate(int nb_threads, int nb_channels, int minimum) {
    int factor = nb_channels;
    if (nb_threads < 4) {
        if (factor != 1 && nb_threads % factor == 0) factor = nb_threads;
        else factor *= nb_threads;
        return ceil_multiple(minimum, factor);
    }
    const int minus_allowed = nb_threads < 8 ? 1 : 3;
    int cand = ceil_multiple(minimum, factor);
    for (;;) {
        const int rem = cand % nb_threads;
        if (rem == 0 || rem >= nb_threads - minus_allowed) return cand;
        cand += factor;
    }
}
}  // namespace

extern "C" int sgpu_stack_blocks(long max_rows, long height, long channels, int nb_threads, int cap,
                                 long *start_row, long *block_height, int *channel, int *nb_blocks,
                                 long *largest) {
    if (nb_threads < 1 || max_rows < 1 || height < 1 || channels < 1 || !nb_blocks)
        return fail(SGPU_GENERIC_ERROR, "block plan: bad threads, rows or size");
    int cand = nb_threads;
    while ((max_rows * cand) / nb_threads < height * channels) cand++;
    cand = refine_candidate(nb_threads, channels == 3 ? 3 : 1, cand);
    *nb_blocks = cand;
    if (cand > cap || !start_row || !block_height || !channel) return fail(SGPU_BAD_ARGUMENT, "block plan: cap");
    const long hb = height * channels / cand;
    long rem = height % (cand / channels);
    long ch = 0, row = 0, big = 0;
    int j = 0;
    do {
        if (j >= cand) return fail(SGPU_GENERIC_ERROR, "block plan: rows left after the last block");
        channel[j] = (int)ch;
        start_row[j] = row;
        long end = row + hb - 1;
        if (rem > 0) {       // one row of the remainder to each first block
            end++;
            rem--;
        }
        if (end >= height - 1 || height - end < hb / 10) {   // end of the channel, or close to it
            end = height - 1;
            row = 0;
            ch++;
            rem = height - (cand / channels * hb);
        } else {
            row = end + 1;
        }
        block_height[j] = end - start_row[j] + 1;
        big = std::max(big, block_height[j]);
        j++;
    } while (ch < channels);
    if (j != cand) return fail(SGPU_GENERIC_ERROR, "block plan: fewer blocks than planned");
    if (largest) *largest = big;
    return SGPU_OK;
}

namespace {
int stack_seq_impl(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params, int use_registration,
                   int use_32bit_output, const char *out_path, uint64_t counts[2], const sgpu_stack_seq_options *opts);
}

extern "C" int sgpu_release_seq_buffers(sgpu_context *ctx) {
    if (!ctx) return fail(SGPU_BAD_ARGUMENT, "null context");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(SGPU_NO_DEVICE, "hipSetDevice failed");
    // the buffers' last users are stream-ordered on the context's streams
    if (hipDeviceSynchronize() != hipSuccess) return fail(SGPU_NO_DEVICE, "hipDeviceSynchronize failed");
    for (sgpu_host::DevBuf *b : {&ctx->seq_in[0], &ctx->seq_in[1], &ctx->seq_out, &ctx->seq_lo, &ctx->seq_hi, &ctx->seq_cnt})
        b->release();
    ctx->seq_pin[0].release();
    ctx->seq_pin[1].release();
    ctx->seq_res.release();
    return SGPU_OK;
}

extern "C" int sgpu_set_seq_readers(sgpu_context *ctx, int readers) {
    if (!ctx || readers < 0) return fail(SGPU_BAD_ARGUMENT, "readers >= 0");
    ctx->seq_readers = readers;
    return SGPU_OK;
}

extern "C" int sgpu_last_seq_stats(sgpu_context *ctx, double out[12]) {
    if (!ctx || !out) return fail(SGPU_BAD_ARGUMENT, "null argument");
    for (int i = 0; i < 12; i++) out[i] = ctx->seq_stats[i];
    return SGPU_OK;
}

extern "C" int sgpu_stack_seq_opts(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                                   int use_registration, int use_32bit_output, const char *out_path,
                                   uint64_t counts[2], const sgpu_stack_seq_options *opts) {
    if (!ctx || !seq_path || !params || !out_path || !opts) return fail(SGPU_BAD_ARGUMENT, "null argument");
    // the source bit depth is this call's: the context's setting is restored
    // on every exit, so a later sgpu_stack_rows_u16 with output_norm is not
    // scaled for an 8-bit sequence stacked earlier
    const int saved_bitpix = ctx->in_bitpix;
    const int r = stack_seq_impl(ctx, seq_path, params, use_registration, use_32bit_output, out_path, counts, opts);
    ctx->in_bitpix = saved_bitpix;
    return r;
}

namespace {
int stack_seq_impl(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params, int use_registration,
                   int use_32bit_output, const char *out_path, uint64_t counts[2], const sgpu_stack_seq_options *opts) {
    const sgpu_stack_seq_options &O = *opts;
    const auto t_entry = std::chrono::steady_clock::now();
    for (double &v : ctx->seq_stats) v = 0.0;
    int rejmaps = O.rejmaps;
    const int lite_norm = O.lite_norm;
    const long max_block_bytes = O.max_block_bytes;
    if (rejmaps < 0 || rejmaps > 2) return fail(SGPU_BAD_ARGUMENT, "rejmaps: 0 none, 1 merged, 2 low and high");
    if (O.feather < 0) return fail(SGPU_BAD_ARGUMENT, "-feather= distance must be >= 0");
    Seq q;
    if (int r = read_seq(seq_path, q)) return r;
    std::vector<Img> all;
    if (int r = open_frames(q, all)) return r;
    // image_indices: every frame passing the filters, in sequence order
    // (stack_one_seq -> convert_parsed_filter_to_filter / setup_filtered_data;
    // no filter = seq_filter_all, -filter-incl = the .seq's included frames)
    std::vector<int> idx;
    if (int r = select_frames(q, O, idx)) return r;
    const int N = (int)idx.size();
    // args->ref_image: sequence_find_refimage, replaced by the first selected
    // frame when filtered out (stack_fill_list_of_unfiltered_images :340-352)
    int refi = find_refimage(q);
    int ref = -1;
    for (int k = 0; k < N; k++)
        if (idx[k] == refi) ref = k;
    if (ref < 0) {
        ref = 0;
        refi = idx[0];
    }
    std::vector<Img> fr(N);
    for (int k = 0; k < N; k++) {
        if (q.type) fr[k] = all[idx[k]];
        else if (int r = fits_open(frame_path(q, q.filenum[idx[k]]).c_str(), fr[k])) return r;
        if (fr[k].w != fr[0].w || fr[k].h != fr[0].h || fr[k].bitpix != fr[0].bitpix ||
            fr[k].nlayers != fr[0].nlayers)
            return fail(SGPU_SEQUENCE_ERROR, "frames differ in size or type");
    }
    const long Win = fr[0].w, Hin = fr[0].h;
    const int NL = fr[0].nlayers;
    const bool u16 = fr[0].bitpix == 16;
    const int es = u16 ? 2 : 4;
    // BYTE_IMG sources (8-bit FITS, 8-bit SER) live in WORD buffers; the
    // sample type still drives normalize_to16bit (median_and_mean.c:547-555,
    // 1729-1732) and the type of a 16-bit result (:1326-1330: an 8-bit stack
    // without output_norm stays BYTE_IMG)
    const bool src8 = fr[0].kind == K_SER ? fr[0].ser_depth == 1 : fr[0].file_bitpix == 8;
    if (int r = sgpu_set_input_bitpix(ctx, src8 ? 8 : fr[0].bitpix)) return r;
    const int reglayer = use_registration ? registration_layer(q) : -1;
    sgpu_stack_params p = *params;
    // -maximize (stack_one_seq :11667-11695): mean stacks of registered
    // sequences; the canvas is the union of the shifted frames
    // (stack_open_all_files, median_and_mean.c:160-190)
    const bool maximize = O.maximize && reglayer >= 0 && p.method == SGPU_METHOD_MEAN;
    // -overlap_norm only with -maximize framing (command.c:11696-11699)
    const bool overlap = O.overlap_norm && maximize && p.normalize != SGPU_NO_NORM;
    long W = Win, H = Hin;
    // args->offset (:182-194): the canvas origin with -maximize, else the
    // reference image's shift truncated to int (FITS sequences; SER keeps 0)
    double off_x = 0.0, off_y = 0.0;
    if (reglayer >= 0) {
        if (maximize) {
            double xmin = DBL_MAX, ymin = DBL_MAX, xmax = -DBL_MAX, ymax = -DBL_MAX;
            for (int k = 0; k < N; k++) {
                const double h02 = q.dx[reglayer][idx[k]], h12 = -q.dy[reglayer][idx[k]];
                xmin = (xmin > h02) ? h02 : xmin;
                ymin = (ymin > h12) ? h12 : ymin;
                xmax = (xmax < h02 + Win) ? h02 + Win : xmax;
                ymax = (ymax < h12 + Hin) ? h12 + Hin : ymax;
            }
            W = (long)((int)xmax - (int)xmin + 1);
            H = (long)((int)ymax - (int)ymin + 1);
            off_x = (int)xmin;
            off_y = -(int)ymin;
        } else if (fr[0].kind != K_SER) {
            off_x = (int)q.dx[reglayer][refi];
            off_y = (int)q.dy[reglayer][refi];
        }
    }
    std::vector<int> shiftx(N, 0), shifty(N, 0);
    bool any_x = false;
    for (int k = 0; k < N && reglayer >= 0; k++) {
        shiftx[k] = round_to_int(q.dx[reglayer][idx[k]] - off_x);
        shifty[k] = round_to_int(q.dy[reglayer][idx[k]] - off_y);
        any_x = any_x || shiftx[k] != 0;
    }
    if (maximize) {
        if (p.shiftx) return fail(SGPU_BAD_ARGUMENT, "-maximize with explicit x shifts");
        any_x = false;                   // placed by the reader
        // the canvas is H rows high: internal row Y of the canvas reads the
        // frame's internal row Y + shifty and is written at FITS row H-1-Y
        // (median_and_mean.c:1597), the frame's internal row y is its FITS
        // row Hin-1-y: in FITS rows the frame is read shifty + H - Hin lower
        for (int k = 0; k < N; k++) shifty[k] += (int)(H - Hin);
    }
    if (any_x && !p.shiftx) p.shiftx = shiftx.data();
    if (rejmaps && (p.method != SGPU_METHOD_MEAN || p.type_of_rejection == SGPU_NO_REJEC))
        rejmaps = 0;   // command.c:11592-11597: maps only with rejection stacking
    // frame weights (-weight=, stack_one_seq :11661, median_and_mean.c:1520-1539)
    std::vector<double> wts;
    int weighting = p.method == SGPU_METHOD_MEAN ? O.weighting : SGPU_NO_WEIGHT;
    if (weighting == SGPU_NOISE_WEIGHT && (p.normalize == SGPU_NO_NORM || overlap))
        weighting = SGPU_NO_WEIGHT;       // :11700-11707, weights ignored
    const bool noise_w = weighting == SGPU_NOISE_WEIGHT;   // per layer, after the normalization pass
    if (weighting == SGPU_WFWHM_WEIGHT || weighting == SGPU_NBSTARS_WEIGHT) {
        if (int r = frame_weights(q, reglayer, idx, weighting, wts)) return r;
    } else if (weighting == SGPU_NBSTACK_WEIGHT && fr[0].kind != K_SER) {
        wts.resize(N);                    // STACKCNT of each frame (:150-159)
        for (int k = 0; k < N; k++) wts[k] = (double)fr[k].stackcnt;
    }
    if (!wts.empty() && !p.weights) p.weights = wts.data();
    // normalization coefficients per layer (coeff.p*[layer])
    const bool do_norm = p.normalize != SGPU_NO_NORM && !p.scale && !p.offset && !p.mul;
    if (noise_w && !do_norm)
        return fail(SGPU_BAD_ARGUMENT, "-weight=noise needs the normalization pass (explicit coefficients given)");
    std::vector<std::vector<double>> n_off(NL), n_mul(NL), n_scl(NL), bg(NL), wl(NL);
    if (do_norm && overlap) {
        // compute_normalization_overlaps (normalization.c:666-906): every pair
        // of the selected frames on their overlap (the registration layer's
        // translations), then the per-layer LU solves; all frames of a layer
        // are resident in HBM together
        const long npix = Win * Hin;
        std::vector<double> h02(N), h12(N);
        for (int k = 0; k < N; k++) {
            h02[k] = q.dx[reglayer][idx[k]];
            h12[k] = -q.dy[reglayer][idx[k]];
        }
        const size_t npairs = (size_t)N * (N - 1) / 2;
        std::vector<long> nij(npairs);
        std::vector<double> tab(npairs * 8);
        std::vector<unsigned char> all((size_t)N * npix * es), tmp;
        void *d_all = nullptr;
        if (hipMalloc(&d_all, all.size()) != hipSuccess) return fail(SGPU_ALLOC_ERROR, "hipMalloc failed (overlaps)");
        int r = SGPU_OK;
        for (int l = 0; l < NL && !r; l++) {
            for (int k = 0; k < N && !r; k++) r = read_rows(fr[k], l, 0, Hin, all.data() + (size_t)k * npix * es, tmp,
                                                            READ_WHOLE);
            if (r) break;
            if (hipMemcpy(d_all, all.data(), all.size(), hipMemcpyHostToDevice) != hipSuccess) {
                r = fail(SGPU_NO_DEVICE, "hipMemcpy failed (overlaps)");
                break;
            }
            r = u16 ? sgpu_overlap_stats_u16_device(ctx, (const uint16_t *)d_all, N, Win, Hin, npix, h02.data(),
                                                    h12.data(), lite_norm, nij.data(), tab.data())
                    : sgpu_overlap_stats_device(ctx, (const float *)d_all, N, Win, Hin, npix, h02.data(), h12.data(),
                                                lite_norm, nij.data(), tab.data());
            if (r) break;
            n_off[l].resize(N);
            n_mul[l].resize(N);
            n_scl[l].resize(N);
            r = sgpu_overlap_factors(p.normalize, lite_norm, N, ref, nij.data(), tab.data(), n_off[l].data(),
                                     n_mul[l].data(), n_scl[l].data());
        }
        (void)hipFree(d_all);
        if (r) return r;
    } else if (do_norm) {
        const long npix = Win * Hin;
        const int batch = (int)std::max(1L, std::min((long)N, (1L << 30) / (npix * es)));
        std::vector<unsigned char> whole((size_t)batch * npix * es);
        std::vector<unsigned char> tmp;
        std::vector<std::vector<double>> stats(NL);
        for (int l = 0; l < NL; l++) {
            stats[l].resize((size_t)4 * N);
            if (noise_w) bg[l].resize(N);
            std::vector<int> status(N, 0);
            for (int f0 = 0; f0 < N; f0 += batch) {
                const int nb = std::min(batch, N - f0);
                for (int k = 0; k < nb; k++)
                    if (int r = read_rows(fr[f0 + k], l, 0, Hin, whole.data() + (size_t)k * npix * es, tmp, READ_WHOLE))
                        return r;
                const int r = u16 ? sgpu_norm_stats_u16(ctx, (const uint16_t *)whole.data(), nb, npix, npix,
                                                        lite_norm, stats[l].data() + 4 * f0, nullptr, status.data() + f0)
                                  : sgpu_norm_stats(ctx, (const float *)whole.data(), nb, npix, npix, lite_norm,
                                                    stats[l].data() + 4 * f0, nullptr, status.data() + f0);
                if (r) return r;
                // imstats bgnoise of the same frames (STATS_NORM includes
                // STATS_BASIC: statistics_float.c:381-400), for -weight=noise
                if (noise_w) {
                    const int rn = u16 ? sgpu_bgnoise_u16(ctx, (const uint16_t *)whole.data(), nb, (int)Win, (int)Hin,
                                                          npix, bg[l].data() + f0)
                                       : sgpu_bgnoise(ctx, (const float *)whole.data(), nb, (int)Win, (int)Hin, npix,
                                                      bg[l].data() + f0);
                    if (rn) return rn;
                }
            }
            for (int k = 0; k < N; k++)
                if (status[k])
                    return fail(SGPU_GENERIC_ERROR, "Normalization failed. Check image " +
                                                        std::to_string(idx[k] + 1) + " first.");
        }
        // -rgb_equal (normalization.c:157-159): every layer against the
        // reference image's estimators of the registration layer (1 when
        // none); a layer the frames do not have keeps its own
        int reflayer_eq = reglayer > -1 ? reglayer : 1;
        if (reflayer_eq >= NL) reflayer_eq = -1;
        for (int l = 0; l < NL; l++) {
            n_off[l].resize(N);
            n_mul[l].resize(N);
            n_scl[l].resize(N);
            const double *rs = (O.equalize_rgb && reflayer_eq >= 0) ? stats[reflayer_eq].data() : nullptr;
            if (int r = sgpu_norm_factors(p.normalize, lite_norm, N, ref, stats[l].data(), rs, n_off[l].data(),
                                          n_mul[l].data(), n_scl[l].data()))
                return r;
            // compute_noise_weights (median_and_mean.c:1111-1135): 1 / (pscale^2
            // bgnoise^2), normalised to a mean of 1, per layer
            if (noise_w) {
                wl[l].resize(N);
                double norm = 0.0;
                for (int k = 0; k < N; k++) {
                    wl[l][k] = 1.f / (n_scl[l][k] * n_scl[l][k] * bg[l][k] * bg[l][k]);
                    norm += wl[l][k];
                }
                norm /= (double)N;
                for (int k = 0; k < N; k++) wl[l][k] /= norm;
            }
        }
    }
    // feathering (args->feather_dist > 0, mean stacks): the masks of every
    // frame (compute_masks, blending.c:199), then per block the ramped mask
    // planes of stack_read_block_data (median_and_mean.c:483-525), which
    // depend on Siril's block plan (stack_compute_parallel_blocks)
    const bool feather = O.feather > 0 && p.method == SGPU_METHOD_MEAN;
    // row blocks in FITS row order: (first row, rows)
    std::vector<std::pair<long, long>> plan;
    long rows = 0;
    if (feather) {
        const int nth_plan = O.block_threads > 0 ? O.block_threads : 1;
        const long max_rows = O.block_max_rows > 0 ? O.block_max_rows : H * NL;
        int nb = 0;
        long largest = 0;
        (void)sgpu_stack_blocks(max_rows, H, NL, nth_plan, 0, nullptr, nullptr, nullptr, &nb, nullptr);
        if (nb < 1) return fail(SGPU_GENERIC_ERROR, "block plan failed");
        std::vector<long> bs(nb), bh(nb);
        std::vector<int> bc(nb);
        if (int r = sgpu_stack_blocks(max_rows, H, NL, nth_plan, nb, bs.data(), bh.data(), bc.data(), &nb, &largest))
            return r;
        // the blocks of one channel (every channel has the same rows), the
        // reference's internal row s is FITS row H - 1 - s
        for (int j = nb - 1; j >= 0; j--)
            if (bc[j] == 0) plan.emplace_back(H - bs[j] - bh[j], bh[j]);
        // a block under 10 rows has an empty downscaled mask area: the
        // reference then keeps whatever its thread's mask buffer held from an
        // earlier block (median_and_mean.c:498-499), this engine writes
        // zero weights -- said once per such stack
        for (const auto &b : plan)
            if (b.second < 10) {
                std::fprintf(stderr, "siril_amd: -feather= block of %ld rows (< 10): its mask weights are 0 here, "
                                     "the reference reuses an earlier block's buffer\n", b.second);
                break;
            }
        rows = largest;
    } else {
        // block height: N frames of `rows` rows within the budget (two buffers)
        const long budget = max_block_bytes > 0 ? max_block_bytes : (512L << 20);
        rows = std::max(1L, budget / ((long)N * W * es));
        rows = std::min(rows, H);
        // the first block's read is the one nothing overlaps: a quarter-size
        // first block shortens it (blocks are independent row ranges, the
        // result does not depend on the plan)
        long r0 = 0;
        if (H > rows && rows >= 4) {
            plan.emplace_back(0, rows / 4);
            r0 = rows / 4;
        }
        for (; r0 < H; r0 += rows) plan.emplace_back(r0, std::min(rows, H - r0));
    }
    const size_t blk = (size_t)N * rows * W * es;
    // block buffers: page-locked (hipHostMalloc) so the H2D copy runs at the
    // link's DMA rate and overlaps the readers of the next block (round 5);
    // pageable vectors when the pinned allocation fails
    std::vector<unsigned char> pageable[2];
    unsigned char *hb[2];
    bool pinned = true;
    HIP_TRY(hipSetDevice(ctx->device));
    for (int b = 0; b < 2; b++) {
        if (ctx->seq_pin[b].ensure(blk) != SGPU_OK) {
            pinned = false;
            pageable[b].resize(blk);
            hb[b] = pageable[b].data();
        } else {
            hb[b] = (unsigned char *)ctx->seq_pin[b].p;
        }
    }
    int read_err[2] = {0, 0};
    // frames of a block are read by a pool of host threads (file reads + byte
    // swaps): the context's setting, else OMP_NUM_THREADS, else 8 (at most 64)
    int nth_cfg = ctx->seq_readers;
    if (nth_cfg <= 0) {
        const char *e = std::getenv("OMP_NUM_THREADS");
        nth_cfg = e && std::atoi(e) > 0 ? std::atoi(e) : 8;
    }
    const int nth = std::max(1, std::min(N, std::min(nth_cfg, 64)));
    double read_wall = 0.0;              // sum over blocks of the readers' wall time
    auto read_block = [&](int slot, int layer, long r0, long nr) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<int> errs(nth, 0);
        auto part = [&](int t) {
            std::vector<unsigned char> tmp, rows_in;
            for (int k = t; k < N && !errs[t]; k += nth) {
                unsigned char *dst = hb[slot] + (size_t)k * nr * W * es;
                if (!maximize) {
                    errs[t] = read_rows(fr[k], layer, r0 - shifty[k], nr, dst, tmp, READ_PARTIAL);
                } else {
                    // rearrange_block_data: the frame's rows into canvas-wide rows
                    rows_in.resize((size_t)nr * Win * es);
                    errs[t] = read_rows(fr[k], layer, r0 - shifty[k], nr, rows_in.data(), tmp, READ_PARTIAL);
                    if (!errs[t]) place_rows(rows_in.data(), Win, dst, W, nr, shiftx[k], es);
                }
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < nth; t++) pool.emplace_back(part, t);
        part(0);
        for (std::thread &th : pool) th.join();
        for (int e : errs)
            if (e && !read_err[slot]) read_err[slot] = e;
        read_wall += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    const bool out32 = !u16 || use_32bit_output;
    const size_t plane = (size_t)W * H;
    // the result image on the host: a page-locked buffer kept in the context
    // (a fresh 96 MB vector was zeroed and page-faulted on every call: most
    // of the 25 ms before the block loop), also the D2H target of the blocks
    struct Span {
        void *p = nullptr;
        size_t n = 0;
        size_t size() const { return n; }
    };
    struct SpanF : Span {
        float *data() const { return (float *)p; }
    } outf;
    struct SpanW : Span {
        uint16_t *data() const { return (uint16_t *)p; }
    } outw;
    {
        const size_t bytes = plane * NL * (out32 ? 4 : 2);
        if (int r = ctx->seq_res.ensure(bytes)) return r;
        if (out32) {
            outf.p = ctx->seq_res.p;
            outf.n = plane * NL;
        } else {
            outw.p = ctx->seq_res.p;
            outw.n = plane * NL;
        }
    }
    std::vector<uint16_t> rlo(rejmaps ? plane * NL : 0), rhi(rejmaps ? plane * NL : 0);
    uint64_t cnt[2] = {0, 0};
    int rc = SGPU_OK;
    // feathering works on device-resident blocks: the masks stay in HBM
    struct Dev {
        std::vector<void *> p;
        void *get(size_t bytes) {
            void *q = nullptr;
            if (hipMalloc(&q, std::max(bytes, (size_t)256)) != hipSuccess) return nullptr;
            p.push_back(q);
            return q;
        }
        ~Dev() {
            for (void *q : p) (void)hipFree(q);
        }
    } dev;
    float *d_masks = nullptr, *d_planes = nullptr;
    unsigned char *d_blk = nullptr, *d_out = nullptr;
    uint16_t *d_lo = nullptr, *d_hi = nullptr;
    uint64_t *d_cnt = nullptr;
    std::vector<int> shifty_ref, placex;
    if (feather) {
        HIP_TRY(hipSetDevice(ctx->device));
        long mw = 0, mh = 0;
        sgpu_feather_mask_size(Win, Hin, &mw, &mh);
        if (mw < 1 || mh < 1) return fail(SGPU_BAD_ARGUMENT, "-feather= needs frames of at least 10x10 pixels");
        d_masks = (float *)dev.get((size_t)N * mw * mh * sizeof(float));
        d_planes = (float *)dev.get((size_t)N * rows * W * sizeof(float));
        d_blk = (unsigned char *)dev.get(blk);
        d_out = (unsigned char *)dev.get((size_t)rows * W * 4);
        d_lo = (uint16_t *)dev.get((size_t)rows * W * 2);
        d_hi = (uint16_t *)dev.get((size_t)rows * W * 2);
        d_cnt = (uint64_t *)dev.get(2 * sizeof(uint64_t));
        if (!d_masks || !d_planes || !d_blk || !d_out || !d_lo || !d_hi || !d_cnt)
            return fail(SGPU_ALLOC_ERROR, "hipMalloc failed (feathering)");
        HIP_TRY(hipMemset(d_cnt, 0, 2 * sizeof(uint64_t)));
        // compute_mask_image_hook: the green layer of colour frames, else the
        // first, of every whole frame (readfits order = FITS rows)
        const int mlayer = NL == 3 ? 1 : 0;
        const long npix = Win * Hin;
        const int batch = (int)std::max(1L, std::min((long)N, (1L << 30) / (npix * es)));
        std::vector<unsigned char> whole((size_t)batch * npix * es), tmp;
        unsigned char *d_whole = (unsigned char *)dev.get(whole.size());
        if (!d_whole) return fail(SGPU_ALLOC_ERROR, "hipMalloc failed (feathering)");
        for (int f0 = 0; f0 < N; f0 += batch) {
            const int nb = std::min(batch, N - f0);
            for (int k = 0; k < nb; k++)
                if (int r = read_rows(fr[f0 + k], mlayer, 0, Hin, whole.data() + (size_t)k * npix * es, tmp, READ_WHOLE))
                    return r;
            HIP_TRY(hipMemcpy(d_whole, whole.data(), (size_t)nb * npix * es, hipMemcpyHostToDevice));
            if (int r = sgpu_feather_masks_device(ctx, d_whole, es, nb, Win, Hin, npix, d_masks + (size_t)f0 * mw * mh))
                return r;
        }
        // the reference's y shift (area.y = start_row + shifty): its canvas
        // row s reads the frame's row s + shifty, i.e. FITS row Y reads the
        // frame's FITS row Y + Hin - H - shifty
        if (reglayer >= 0) {
            shifty_ref.resize(N);
            for (int k = 0; k < N; k++) shifty_ref[k] = shifty[k] + (int)(Hin - H);
        }
        if (maximize) placex = shiftx;
    }
    // the non-feathering path (round 5): per block an H2D copy of the pinned
    // buffer on a copy stream (waiting for the stack that last used the
    // device buffer), the stack on the context stream (waiting for the copy),
    // the small outputs back; the readers of the next block run meanwhile
    struct Pipe {
        hipStream_t cs = nullptr;
        hipEvent_t h0[2] = {nullptr, nullptr}, h1[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
        hipEvent_t k0 = nullptr, k1 = nullptr;
        ~Pipe() {
            for (hipEvent_t e : {h0[0], h0[1], h1[0], h1[1], done[0], done[1], k0, k1})
                if (e) (void)hipEventDestroy(e);
            if (cs) (void)hipStreamDestroy(cs);
        }
    } pp;
    unsigned char *d_in[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    double h2d_ms = 0.0, kern_ms = 0.0, h2d_bytes = 0.0;
    int nblocks = 0;
    if (!feather) {
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipStreamCreateWithFlags(&pp.cs, hipStreamNonBlocking));
        for (int b = 0; b < 2; b++) {
            HIP_TRY(hipEventCreate(&pp.h0[b]));
            HIP_TRY(hipEventCreate(&pp.h1[b]));
            HIP_TRY(hipEventCreateWithFlags(&pp.done[b], hipEventDisableTiming));
            if (int r = ctx->seq_in[b].ensure(blk)) return r;
            d_in[b] = (unsigned char *)ctx->seq_in[b].p;
        }
        HIP_TRY(hipEventCreate(&pp.k0));
        HIP_TRY(hipEventCreate(&pp.k1));
        if (int r = ctx->seq_out.ensure((size_t)rows * W * 4)) return r;
        if (int r = ctx->seq_cnt.ensure(2 * sizeof(uint64_t))) return r;
        d_out = (unsigned char *)ctx->seq_out.p;
        d_cnt = (uint64_t *)ctx->seq_cnt.p;
        if (rejmaps) {
            if (int r = ctx->seq_lo.ensure((size_t)rows * W * 2)) return r;
            if (int r = ctx->seq_hi.ensure((size_t)rows * W * 2)) return r;
            d_lo = (uint16_t *)ctx->seq_lo.p;
            d_hi = (uint16_t *)ctx->seq_hi.p;
        }
        HIP_TRY(hipMemsetAsync(d_cnt, 0, 2 * sizeof(uint64_t), ctx->stream));
    }
    std::vector<std::string> hist;
    {
        char h[80];
        std::snprintf(h, sizeof h, "Stacking method: %s (siril_amd MI355X engine)",
                      p.method == SGPU_METHOD_MEDIAN ? "median" : "average with rejection");
        hist.push_back(h);
        std::snprintf(h, sizeof h, "Integration of %d images, rejection %d (%g, %g)", N, p.type_of_rejection,
                      p.sig[0], p.sig[1]);
        hist.push_back(h);
    }
    // the result streams to its file block by block unless -output_norm
    // needs the whole image first (norm_to_0_1_range after the stack)
    const bool stream_out = !(out32 && p.output_norm);
    FitsStream fstream;
    if (stream_out)
        if (int r = fstream.open(out_path, W, H, NL, out32 ? -32 : ((src8 && !p.output_norm) ? 8 : 16), hist))
            return r;
    const void *out_host = out32 ? (const void *)outf.data() : (const void *)outw.data();
    const auto loop_t0 = std::chrono::steady_clock::now();
    for (int l = 0; l < NL && !rc; l++) {
        sgpu_stack_params pl = p;
        if (do_norm) {
            pl.offset = n_off[l].data();
            pl.mul = n_mul[l].data();
            pl.scale = n_scl[l].data();
        }
        if (!wl[l].empty()) pl.weights = wl[l].data();
        read_err[0] = read_err[1] = 0;
        read_block(0, l, plan[0].first, plan[0].second);
        int slot = 0;
        for (size_t b = 0; b < plan.size(); b++) {
            const long r0 = plan[b].first, nr = plan[b].second;
            if (read_err[slot]) {   // (messages of reader threads stay thread-local)
                rc = fail(read_err[slot], "reading a block of the sequence failed");
                break;
            }
            std::thread reader;
            if (!feather) {
                // H2D of this block on the copy stream, after the stack that
                // last read the device buffer
                const size_t nbytes = (size_t)N * nr * W * es;
                if ((used[slot] && hipStreamWaitEvent(pp.cs, pp.done[slot], 0) != hipSuccess) ||
                    hipEventRecord(pp.h0[slot], pp.cs) != hipSuccess ||
                    hipMemcpyAsync(d_in[slot], hb[slot], nbytes, hipMemcpyHostToDevice, pp.cs) != hipSuccess ||
                    hipEventRecord(pp.h1[slot], pp.cs) != hipSuccess) {
                    rc = fail(SGPU_NO_DEVICE, "H2D copy of a sequence block failed");
                    break;
                }
                h2d_bytes += (double)nbytes;
                // the other host buffer is free once its own copy is through
                if (used[slot ^ 1] && hipEventSynchronize(pp.h1[slot ^ 1]) != hipSuccess) {
                    rc = fail(SGPU_NO_DEVICE, "H2D copy of a sequence block failed");
                    break;
                }
            }
            if (b + 1 < plan.size()) reader = std::thread(read_block, slot ^ 1, l, plan[b + 1].first, plan[b + 1].second);
            const size_t o = l * plane + (size_t)r0 * W;
            uint16_t *lo = rejmaps ? rlo.data() + o : nullptr, *hi = rejmaps ? rhi.data() + o : nullptr;
            if (feather) {
                const size_t n = (size_t)nr * W;
                rc = sgpu_feather_block_device(ctx, d_masks, N, Win, Hin, H - r0 - nr, nr,
                                               shifty_ref.empty() ? nullptr : shifty_ref.data(),
                                               placex.empty() ? nullptr : placex.data(), W, (float)O.feather, 1,
                                               d_planes, (long)n);
                if (!rc && hipMemcpyAsync(d_blk, hb[slot], (size_t)N * n * es, hipMemcpyHostToDevice,
                                          ctx->stream) != hipSuccess)
                    rc = fail(SGPU_NO_DEVICE, "hipMemcpy failed (feathering)");
                if (!rc && u16)
                    rc = sgpu_stack_rows_u16_planes_device(ctx, (const uint16_t *)d_blk, nullptr, d_planes, N, W, nr,
                                                           (long)n, &pl, out32 ? (float *)d_out : nullptr,
                                                           out32 ? nullptr : (uint16_t *)d_out, rejmaps ? d_lo : nullptr,
                                                           rejmaps ? d_hi : nullptr, d_cnt);
                else if (!rc)
                    rc = sgpu_stack_rows_planes_device(ctx, (const float *)d_blk, nullptr, d_planes, N, W, nr, (long)n,
                                                       &pl, (float *)d_out, rejmaps ? d_lo : nullptr,
                                                       rejmaps ? d_hi : nullptr, d_cnt);
                if (!rc) {
                    hipError_t e = out32 ? hipMemcpyAsync(outf.data() + o, d_out, n * 4, hipMemcpyDeviceToHost, ctx->stream)
                                         : hipMemcpyAsync(outw.data() + o, d_out, n * 2, hipMemcpyDeviceToHost, ctx->stream);
                    if (e == hipSuccess && rejmaps)
                        e = hipMemcpyAsync(lo, d_lo, n * 2, hipMemcpyDeviceToHost, ctx->stream);
                    if (e == hipSuccess && rejmaps)
                        e = hipMemcpyAsync(hi, d_hi, n * 2, hipMemcpyDeviceToHost, ctx->stream);
                    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
                    if (e != hipSuccess) rc = fail(SGPU_NO_DEVICE, "hipMemcpy failed (feathering)");
                    else if (stream_out) fstream.emit(out_host, o, n);
                }
            } else {
                const size_t n = (size_t)nr * W;
                if (hipStreamWaitEvent(ctx->stream, pp.h1[slot], 0) != hipSuccess ||
                    hipEventRecord(pp.k0, ctx->stream) != hipSuccess)
                    rc = fail(SGPU_NO_DEVICE, "stream ordering failed");
                if (!rc && u16)
                    rc = sgpu_stack_rows_u16_device(ctx, (const uint16_t *)d_in[slot], N, W, nr, (long)n, &pl,
                                                    out32 ? (float *)d_out : nullptr,
                                                    out32 ? nullptr : (uint16_t *)d_out, d_lo, d_hi, d_cnt);
                else if (!rc)
                    rc = sgpu_stack_rows_device(ctx, (const float *)d_in[slot], N, W, nr, (long)n, &pl,
                                                (float *)d_out, d_lo, d_hi, d_cnt);
                if (!rc) {
                    hipError_t e = hipEventRecord(pp.k1, ctx->stream);
                    if (e == hipSuccess) e = hipEventRecord(pp.done[slot], ctx->stream);
                    used[slot] = true;
                    if (e == hipSuccess)
                        e = out32 ? hipMemcpyAsync(outf.data() + o, d_out, n * 4, hipMemcpyDeviceToHost, ctx->stream)
                                  : hipMemcpyAsync(outw.data() + o, d_out, n * 2, hipMemcpyDeviceToHost, ctx->stream);
                    if (e == hipSuccess && rejmaps) e = hipMemcpyAsync(lo, d_lo, n * 2, hipMemcpyDeviceToHost, ctx->stream);
                    if (e == hipSuccess && rejmaps) e = hipMemcpyAsync(hi, d_hi, n * 2, hipMemcpyDeviceToHost, ctx->stream);
                    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
                    float a = 0.f, k = 0.f;
                    if (e == hipSuccess) e = hipEventElapsedTime(&a, pp.h0[slot], pp.h1[slot]);
                    if (e == hipSuccess) e = hipEventElapsedTime(&k, pp.k0, pp.k1);
                    h2d_ms += a;
                    kern_ms += k;
                    nblocks++;
                    if (e != hipSuccess) rc = fail(SGPU_NO_DEVICE, "sequence block stack failed");
                    else if (stream_out) fstream.emit(out_host, o, n);
                }
            }
            if (reader.joinable()) reader.join();
            if (rc) break;
            slot ^= 1;
        }
    }
    ctx->seq_stats[0] = nblocks;
    ctx->seq_stats[1] = read_wall;
    ctx->seq_stats[2] = h2d_ms;
    ctx->seq_stats[3] = h2d_bytes;
    ctx->seq_stats[4] = kern_ms;
    ctx->seq_stats[5] = std::chrono::duration<double>(std::chrono::steady_clock::now() - loop_t0).count();
    ctx->seq_stats[6] = pinned ? 1.0 : 0.0;
    ctx->seq_stats[7] = nth;
    if (!rc && d_cnt) {
        uint64_t dc[2];
        if (hipMemcpy(dc, d_cnt, sizeof dc, hipMemcpyDeviceToHost) != hipSuccess)
            return fail(SGPU_NO_DEVICE, "hipMemcpy failed (feathering)");
        cnt[0] += dc[0];
        cnt[1] += dc[1];
    }
    if (rc) return rc;
    if (out32 && p.output_norm) {
        // norm_to_0_1_range (median_and_mean.c:557-582, called at :1774-1775)
        // on the assembled image (all layers), on the device (output_norm.hip)
        const size_t bytes = outf.size() * sizeof(float);
        if (int r = ctx->out.ensure(bytes)) return r;
        HIP_TRY(hipMemcpyAsync(ctx->out.p, outf.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
        if (int r = sgpu_norm_to_0_1_range_device(ctx, (float *)ctx->out.p, (long)outf.size())) return r;
        HIP_TRY(hipMemcpyAsync(outf.data(), ctx->out.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    if (counts) {
        counts[0] = cnt[0];
        counts[1] = cnt[1];
    }
    const auto t_write = std::chrono::steady_clock::now();
    const auto secs = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    };
    ctx->seq_stats[8] = std::chrono::duration<double>(loop_t0 - t_entry).count();
    int wr = stream_out ? fstream.close()
             : out32    ? fits_write(out_path, outf.data(), W, H, NL, -32, hist)
                        : fits_write(out_path, outw.data(), W, H, NL, (src8 && !p.output_norm) ? 8 : 16, hist);
    ctx->seq_stats[9] = secs(t_write);
    ctx->seq_stats[10] = secs(t_entry);
    if (wr || !rejmaps) return wr;
    // rejection maps (command.c:11778-11803): soper_unscaled_div_ushort_to_float
    // (core/arithm.c:128-145): count * (1.0f / (float)N), saved as float images
    const float op = 1.0f / (float)N;
    std::vector<float> m(plane * NL);
    if (rejmaps == 1) {
        for (size_t i = 0; i < m.size(); i++) {
            const unsigned t = (unsigned)rlo[i] + rhi[i];   // truncate_to_WORD(rej[0] + rej[1])
            m[i] = (float)(t > 65535u ? 65535u : t) * op;
        }
        return fits_write(replace_ext(out_path, "_low+high_rejmap.fit").c_str(), m.data(), W, H, NL, -32, hist);
    }
    for (size_t i = 0; i < m.size(); i++) m[i] = rlo[i] * op;
    if ((wr = fits_write(replace_ext(out_path, "_low_rejmap.fit").c_str(), m.data(), W, H, NL, -32, hist))) return wr;
    for (size_t i = 0; i < m.size(); i++) m[i] = rhi[i] * op;
    return fits_write(replace_ext(out_path, "_high_rejmap.fit").c_str(), m.data(), W, H, NL, -32, hist);
}
}  // namespace
