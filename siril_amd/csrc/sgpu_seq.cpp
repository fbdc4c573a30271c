// sgpu_seq.cpp -- headless sequence stacking: the host side of Siril's
// scripting path `stack <seq> ...` (command.c:11985 process_stackone ->
// stack_one_seq :11729 -> main_stack stacking.c:76 -> stack_mean_or_median
// median_and_mean.c:1261) for regular FITS sequences.
//
//   * .seq reader: io/seqfile.c:84-300 -- S (quoted or bare name, beg,
//     number, selnum, fixed, reference, version, ...), L, I (filenum, incl)
//     and R0 registration lines (v4+: `fwhm wfwhm round quality bkg nstars
//     H h00..h22`; v1-3: shiftx shifty first);
//   * frame names: seqname + %0{fixed}d + extension (io/sequence.c:1335-1352);
//   * FITS: one plane, BITPIX -32 (float, no BSCALE/BZERO scaling) or 16 /
//     BZERO 32768 (DATA_USHORT), big-endian, 2880-byte blocks;
//   * block reader: stack_read_block_data (median_and_mean.c:382-545) in FITS
//     row order -- output row R reads input row R - shifty with zero fill
//     (Siril reads bottom-up, flips, and writes row H-1-y: the net map is the
//     identity on FITS rows, shifted by the registration dy = -h12);
//     the x shift round_to_int(h02) is applied on the device
//     (median_and_mean.c:1615-1636);
//   * compute: sgpu_stack_rows / sgpu_stack_rows_u16 per block, the next
//     block read by a second thread while the GPU stacks the current one;
//   * result: BITPIX -32 (float input or use_32bit_output) or 16 with
//     BZERO 32768, saved like savefits (command.c:11772).
// Normalization (params->normalize != NO_NORM with no coefficient arrays):
// compute_normalization (stacking/normalization.c:249-294) -- each included
// frame is read whole (unshifted) in batches, its estimators computed on the
// GPU (norm_stats.hip, STATS_NORM or STATS_LITENORM) and turned into
// coefficients relative to the reference image (sgpu_norm_factors).  The
// reference image is the .seq's reference_image when valid, else the first
// included frame (sequence_find_refimage io/sequence.c:1791 also ranks
// frames by registration FWHM / quality, which the headless .seq files of
// this engine do not carry).  DATA_FLOAT and DATA_USHORT sequences.
#include <algorithm>
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

// ------------------------------------------------------------------ FITS
struct Fits {
    std::string path;
    long w = 0, h = 0;
    int bitpix = 0;
    double bzero = 0.0, bscale = 1.0;
    long data_off = 0;
    bool has_datamax = false;   // DATAMAX card present
    double datamax = 0.0;
    bool from_siril = false;    // PROGRAM card contains "Siril" (io/fits_keywords.c:1281)
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

int fits_open(const char *path, Fits &f) {
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return fail(SGPU_SEQUENCE_ERROR, (std::string("cannot open FITS ") + path).c_str());
    f = Fits();
    f.path = path;
    char block[2880];
    long naxis = -1, n3 = 1;
    bool end = false;
    long nblocks = 0;
    while (!end && std::fread(block, 1, 2880, fp) == 2880) {
        nblocks++;
        for (int c = 0; c < 36 && !end; c++) {
            const char *card = block + 80 * c;
            char key[9];
            std::memcpy(key, card, 8);
            key[8] = 0;
            for (int i = 7; i >= 0 && key[i] == ' '; i--) key[i] = 0;
            if (!std::strcmp(key, "END")) end = true;
            else if (!std::strcmp(key, "BITPIX")) f.bitpix = (int)card_num(card);
            else if (!std::strcmp(key, "NAXIS")) naxis = (long)card_num(card);
            else if (!std::strcmp(key, "NAXIS1")) f.w = (long)card_num(card);
            else if (!std::strcmp(key, "NAXIS2")) f.h = (long)card_num(card);
            else if (!std::strcmp(key, "NAXIS3")) n3 = (long)card_num(card);
            else if (!std::strcmp(key, "BZERO")) f.bzero = card_num(card);
            else if (!std::strcmp(key, "BSCALE")) f.bscale = card_num(card);
            else if (!std::strcmp(key, "DATAMAX")) {
                const double v = card_num(card);
                if (v == v) {
                    f.has_datamax = true;
                    f.datamax = v;
                }
            } else if (!std::strcmp(key, "PROGRAM")) {
                const char *q0 = (const char *)std::memchr(card + 10, '\'', 70);
                const char *q1 = q0 ? (const char *)std::memchr(q0 + 1, '\'', card + 80 - q0 - 1) : nullptr;
                f.from_siril = q0 && q1 && std::string(q0 + 1, q1).find("Siril") != std::string::npos;
            }
        }
    }
    std::fclose(fp);
    if (!end) return fail(SGPU_SEQUENCE_ERROR, (std::string("no END card in ") + path).c_str());
    if (naxis < 2 || n3 != 1 || f.w < 1 || f.h < 1)
        return fail(SGPU_SEQUENCE_ERROR, "only single-plane 2-D FITS images are supported");
    if (f.bitpix == -32) {
        // Siril renormalises scaled float data (image_format_fits.c:988-1007)
        if (f.bzero != 0.0 || f.bscale != 1.0)
            return fail(SGPU_SEQUENCE_ERROR, "scaled float FITS (BZERO/BSCALE) is not supported");
    } else if (f.bitpix == 16) {
        // unsigned convention (BZERO 32768) and plain signed shorts both read
        // as DATA_USHORT stored + 32768 (src/tests/fits_scaling_test.c:190-205,
        // :317-332); physical float scaling of 16-bit data is not supported
        if (f.bscale != 1.0 || (f.bzero != 32768.0 && f.bzero != 0.0))
            return fail(SGPU_SEQUENCE_ERROR, "scaled 16-bit FITS (BSCALE/BZERO) is not supported");
    } else {
        return fail(SGPU_SEQUENCE_ERROR, "FITS BITPIX must be -32 or 16");
    }
    f.data_off = nblocks * 2880;
    return SGPU_OK;
}

inline uint32_t be32(const unsigned char *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// max over all samples of a float file, in float (fit_stats, image_format_fits.c:84-140)
int fits_float_max(const Fits &f, float &mx);

// convert_floats (image_format_fits.c:648-672) for FLOAT_IMG: falls through to
// the USHORT case, data[i] * INV_USHRT_MAX_SINGLE in float
inline void convert_floats(float *d, size_t n) {
    for (size_t i = 0; i < n; i++) d[i] = d[i] * 0.000015259022f;   // INV_USHRT_MAX_SINGLE
}

// rows [r0, r0+n) of the image in FITS order into dst (float or WORD per
// element, row-major, width w); rows outside [0, h) are zero-filled.
// Float files are brought to [0, 1] like Siril reads them (mode):
//  READ_PARTIAL: DATAMAX card, or when absent the max of the 3 (or 4)
//    samples dest[0], dest[n/3], ... of the region actually read (the rows
//    inside the image), `> 10` -> convert_floats (image_format_fits.c:994-1007);
//  READ_WHOLE: keywords.data_max, which is the file's true max for files not
//    written by Siril (fits_keywords.c:1281-1288) and DATAMAX (or 0) otherwise,
//    `> 10` -> convert_floats (:906-910).
int fits_read_rows(const Fits &f, long r0, long n, void *dst, std::vector<unsigned char> &tmp,
                   int mode = READ_RAW) {
    const int es = f.bitpix == -32 ? 4 : 2;
    std::memset(dst, 0, (size_t)n * f.w * es);
    const long a = std::max(r0, 0L), b = std::min(r0 + n, f.h);
    if (a >= b) return SGPU_OK;
    FILE *fp = std::fopen(f.path.c_str(), "rb");
    if (!fp) return fail(SGPU_SEQUENCE_ERROR, (std::string("cannot open FITS ") + f.path).c_str());
    const size_t bytes = (size_t)(b - a) * f.w * es;
    tmp.resize(bytes);
    if (std::fseek(fp, f.data_off + (long)((size_t)a * f.w * es), SEEK_SET) != 0 ||
        std::fread(tmp.data(), 1, bytes, fp) != bytes) {
        std::fclose(fp);
        return fail(SGPU_SEQUENCE_ERROR, (std::string("short read in ") + f.path).c_str());
    }
    std::fclose(fp);
    const size_t cnt = (size_t)(b - a) * f.w;
    if (es == 4) {
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
    } else {
        uint16_t *o = (uint16_t *)dst + (size_t)(a - r0) * f.w;
        for (size_t i = 0; i < cnt; i++)   // signed big-endian + BZERO 32768
            o[i] = (uint16_t)((((uint16_t)tmp[2 * i] << 8) | tmp[2 * i + 1]) ^ 0x8000u);
    }
    return SGPU_OK;
}

int fits_float_max(const Fits &f, float &mx) {
    mx = -1.E33f;
    std::vector<unsigned char> tmp;
    const long step = std::max(1L, (64L << 20) / (f.w * 4));
    std::vector<float> chunk;
    for (long r = 0; r < f.h; r += step) {
        const long nr = std::min(step, f.h - r);
        chunk.resize((size_t)nr * f.w);
        if (int e = fits_read_rows(f, r, nr, chunk.data(), tmp, READ_RAW)) return e;
        for (float v : chunk) mx = (v > mx) ? v : mx;
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

int fits_write(const char *path, const void *data, long w, long h, int bitpix,
               const std::vector<std::string> &history) {
    std::string hdr;
    put_card(hdr, "SIMPLE", "T", "conforms to FITS standard");
    put_card(hdr, "BITPIX", std::to_string(bitpix), "array data type");
    put_card(hdr, "NAXIS", "2", "number of array dimensions");
    put_card(hdr, "NAXIS1", std::to_string(w));
    put_card(hdr, "NAXIS2", std::to_string(h));
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
    FILE *fp = std::fopen(path, "wb");
    if (!fp) return fail(SGPU_GENERIC_ERROR, (std::string("cannot write ") + path).c_str());
    bool ok = std::fwrite(hdr.data(), 1, hdr.size(), fp) == hdr.size();
    const int es = bitpix == -32 ? 4 : 2;
    const size_t cnt = (size_t)w * h;
    std::vector<unsigned char> buf(cnt * es);
    for (size_t i = 0; i < cnt; i++) {
        if (es == 4) {
            const uint32_t u = ((const uint32_t *)data)[i];
            buf[4 * i] = (unsigned char)(u >> 24);
            buf[4 * i + 1] = (unsigned char)(u >> 16);
            buf[4 * i + 2] = (unsigned char)(u >> 8);
            buf[4 * i + 3] = (unsigned char)u;
        } else {
            const uint16_t u = (uint16_t)(((const uint16_t *)data)[i] ^ 0x8000u);
            buf[2 * i] = (unsigned char)(u >> 8);
            buf[2 * i + 1] = (unsigned char)u;
        }
    }
    ok = ok && std::fwrite(buf.data(), 1, buf.size(), fp) == buf.size();
    const size_t pad = (2880 - buf.size() % 2880) % 2880;
    std::vector<unsigned char> zeros(pad, 0);
    ok = ok && std::fwrite(zeros.data(), 1, pad, fp) == pad;
    ok = (std::fclose(fp) == 0) && ok;
    return ok ? SGPU_OK : fail(SGPU_GENERIC_ERROR, (std::string("write failed: ") + path).c_str());
}

// ------------------------------------------------------------------- .seq
struct Seq {
    std::string dir, name;
    int beg = 0, number = 0, selnum = 0, fixed = 0, reference = 0, version = -1;
    std::vector<int> filenum, incl;
    std::vector<double> dx, dy;     // layer-0 registration translation
    bool has_reg = false;
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
    q.dir = slash == std::string::npos ? "" : p.substr(0, slash + 1);
    char line[512];
    int ni = 0, nr = 0;
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
            q.dx.assign(q.number, 0.0);
            q.dy.assign(q.number, 0.0);
            have_s = true;
        } else if (line[0] == 'T') {
            err = fail(SGPU_SEQUENCE_ERROR, "only regular FITS sequences are supported (T line)");
            break;
        } else if (line[0] == 'I' && line[1] == ' ') {
            if (!have_s || ni >= q.number) { err = fail(SGPU_SEQUENCE_ERROR, "bad I line"); break; }
            if (std::sscanf(line + 2, "%d %d", &q.filenum[ni], &q.incl[ni]) != 2) {
                err = fail(SGPU_SEQUENCE_ERROR, "bad I line");
                break;
            }
            ni++;
        } else if (line[0] == 'R' && line[1] == '0') {
            if (!have_s || nr >= q.number) { err = fail(SGPU_SEQUENCE_ERROR, "bad R0 line"); break; }
            if (q.version >= 4) {
                double f[6], H[9];
                int ns;
                if (std::sscanf(line + 3, "%lg %lg %lg %lg %lg %d H %lg %lg %lg %lg %lg %lg %lg %lg %lg", &f[0],
                                &f[1], &f[2], &f[3], &f[4], &ns, &H[0], &H[1], &H[2], &H[3], &H[4], &H[5], &H[6],
                                &H[7], &H[8]) != 15) {
                    err = fail(SGPU_SEQUENCE_ERROR, "bad R0 line");
                    break;
                }
                q.dx[nr] = H[2];       // translation_from_H: dx = h02, dy = -h12
                q.dy[nr] = -H[5];
            } else {
                float sx, sy;
                if (std::sscanf(line + 3, "%f %f", &sx, &sy) != 2) { err = fail(SGPU_SEQUENCE_ERROR, "bad R0 line"); break; }
                q.dx[nr] = sx;         // H_from_translation(shiftx, shifty)
                q.dy[nr] = sy;
            }
            nr++;
            q.has_reg = true;
        }
    }
    std::fclose(fp);
    if (err) return err;
    if (!have_s || ni != q.number) return fail(SGPU_SEQUENCE_ERROR, "sequence file incomplete");
    return SGPU_OK;
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

}  // namespace

extern "C" int sgpu_fits_info(const char *path, long *width, long *height, int *bitpix) {
    if (!path) return fail(SGPU_BAD_ARGUMENT, "null path");
    Fits f;
    if (int r = fits_open(path, f)) return r;
    if (width) *width = f.w;
    if (height) *height = f.h;
    if (bitpix) *bitpix = f.bitpix;
    return SGPU_OK;
}

extern "C" int sgpu_fits_read_rows_ex(const char *path, long row0, long nrows, void *out, int mode) {
    if (!path || !out || nrows < 0 || mode < READ_RAW || mode > READ_WHOLE)
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    Fits f;
    if (int r = fits_open(path, f)) return r;
    std::vector<unsigned char> tmp;
    return fits_read_rows(f, row0, nrows, out, tmp, mode);
}

extern "C" int sgpu_fits_read_rows(const char *path, long row0, long nrows, void *out) {
    return sgpu_fits_read_rows_ex(path, row0, nrows, out, READ_RAW);
}


extern "C" int sgpu_fits_write(const char *path, const void *data, long width, long height, int bitpix) {
    if (!path || !data || width < 1 || height < 1 || (bitpix != -32 && bitpix != 16))
        return fail(SGPU_BAD_ARGUMENT, "bad argument");
    return fits_write(path, data, width, height, bitpix, {});
}

extern "C" int sgpu_stack_seq_ex(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                                 int use_registration, int use_32bit_output, const char *out_path,
                                 uint64_t counts[2], long max_block_bytes, int lite_norm);

extern "C" int sgpu_stack_seq(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                              int use_registration, int use_32bit_output, const char *out_path,
                              uint64_t counts[2], long max_block_bytes) {
    return sgpu_stack_seq_ex(ctx, seq_path, params, use_registration, use_32bit_output, out_path, counts,
                             max_block_bytes, 0);
}

extern "C" int sgpu_stack_seq_ex(sgpu_context *ctx, const char *seq_path, const sgpu_stack_params *params,
                                 int use_registration, int use_32bit_output, const char *out_path,
                                 uint64_t counts[2], long max_block_bytes, int lite_norm) {
    if (!ctx || !seq_path || !params || !out_path) return fail(SGPU_BAD_ARGUMENT, "null argument");
    Seq q;
    if (int r = read_seq(seq_path, q)) return r;
    // image_indices: included frames in sequence order (stack_one_seq filters)
    std::vector<int> idx;
    for (int i = 0; i < q.number; i++)
        if (q.incl[i]) idx.push_back(i);
    const int N = (int)idx.size();
    if (N < 1) return fail(SGPU_SEQUENCE_ERROR, "no image selected in the sequence");
    std::vector<Fits> fr(N);
    for (int k = 0; k < N; k++) {
        if (int r = fits_open(frame_path(q, q.filenum[idx[k]]).c_str(), fr[k])) return r;
        if (fr[k].w != fr[0].w || fr[k].h != fr[0].h || fr[k].bitpix != fr[0].bitpix)
            return fail(SGPU_SEQUENCE_ERROR, "frames differ in size or type");
    }
    const long W = fr[0].w, H = fr[0].h;
    const bool u16 = fr[0].bitpix == 16;
    const int es = u16 ? 2 : 4;
    const bool reg = use_registration && q.has_reg;
    std::vector<int> shiftx(N, 0), shifty(N, 0);
    bool any_x = false;
    for (int k = 0; k < N; k++) {
        if (!reg) break;
        shiftx[k] = round_to_int(q.dx[idx[k]]);
        shifty[k] = round_to_int(q.dy[idx[k]]);
        any_x = any_x || shiftx[k] != 0;
    }
    sgpu_stack_params p = *params;
    if (any_x && !p.shiftx) p.shiftx = shiftx.data();
    std::vector<double> n_off, n_mul, n_scl;
    if (p.normalize != SGPU_NO_NORM && !p.scale && !p.offset && !p.mul) {
        int ref = 0;
        for (int k = 0; k < N; k++)
            if (idx[k] == q.reference) ref = k;
        if (q.reference >= 0 && q.reference < q.number && !q.incl[q.reference])
            return fail(SGPU_GENERIC_ERROR, "The reference image is not in the selected set of images.");
        const long npix = W * H;
        const int batch = (int)std::max(1L, std::min((long)N, (1L << 30) / (npix * es)));
        std::vector<unsigned char> whole((size_t)batch * npix * es);
        std::vector<double> stats((size_t)4 * N);
        std::vector<int> status(N, 0);
        std::vector<unsigned char> tmp;
        for (int f0 = 0; f0 < N; f0 += batch) {
            const int nb = std::min(batch, N - f0);
            for (int k = 0; k < nb; k++)
                if (int r = fits_read_rows(fr[f0 + k], 0, H, whole.data() + (size_t)k * npix * es, tmp,
                                               READ_WHOLE))
                    return r;
            const int r = u16 ? sgpu_norm_stats_u16(ctx, (const uint16_t *)whole.data(), nb, npix, npix, lite_norm,
                                                    stats.data() + 4 * f0, nullptr, status.data() + f0)
                              : sgpu_norm_stats(ctx, (const float *)whole.data(), nb, npix, npix, lite_norm,
                                                stats.data() + 4 * f0, nullptr, status.data() + f0);
            if (r) return r;
        }
        for (int k = 0; k < N; k++)
            if (status[k])
                return fail(SGPU_GENERIC_ERROR, "Normalization failed. Check image " + std::to_string(idx[k] + 1) +
                                                    " first.");
        n_off.resize(N);
        n_mul.resize(N);
        n_scl.resize(N);
        if (int r = sgpu_norm_factors(p.normalize, lite_norm, N, ref, stats.data(), nullptr, n_off.data(),
                                      n_mul.data(), n_scl.data()))
            return r;
        p.offset = n_off.data();
        p.mul = n_mul.data();
        p.scale = n_scl.data();
    }
    // block height: N frames of `rows` rows within the budget (two buffers)
    const long budget = max_block_bytes > 0 ? max_block_bytes : (512L << 20);
    long rows = std::max(1L, budget / ((long)N * W * es));
    rows = std::min(rows, H);
    const size_t blk = (size_t)N * rows * W * es;
    std::vector<unsigned char> buf[2] = {std::vector<unsigned char>(blk), std::vector<unsigned char>(blk)};
    int read_err[2] = {0, 0};
    // frames of a block are read by up to 8 threads (file reads + byte swaps)
    const int nth = std::max(1, std::min(N, 8));
    auto read_block = [&](int slot, long r0, long nr) {
        std::vector<int> errs(nth, 0);
        auto part = [&](int t) {
            std::vector<unsigned char> tmp;
            for (int k = t; k < N && !errs[t]; k += nth)
                errs[t] = fits_read_rows(fr[k], r0 - shifty[k], nr,
                                         buf[slot].data() + (size_t)k * nr * W * es, tmp, READ_PARTIAL);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < nth; t++) pool.emplace_back(part, t);
        part(0);
        for (std::thread &th : pool) th.join();
        for (int e : errs)
            if (e && !read_err[slot]) read_err[slot] = e;
    };
    const bool out32 = !u16 || use_32bit_output;
    std::vector<float> outf(out32 ? (size_t)W * H : 0);
    std::vector<uint16_t> outw(out32 ? 0 : (size_t)W * H);
    uint64_t cnt[2] = {0, 0};
    long r0 = 0;
    long nr = std::min(rows, H);
    read_block(0, 0, nr);
    int slot = 0, rc = SGPU_OK;
    while (r0 < H) {
        if (read_err[slot]) {   // (messages of reader threads stay thread-local)
            rc = fail(read_err[slot], "reading a FITS block of the sequence failed");
            break;
        }
        const long nxt = r0 + nr, nnr = std::min(rows, H - nxt);
        std::thread reader;
        if (nxt < H) reader = std::thread(read_block, slot ^ 1, nxt, nnr);
        if (u16)
            rc = sgpu_stack_rows_u16(ctx, (const uint16_t *)buf[slot].data(), N, W, nr, nr * W, &p,
                                     out32 ? outf.data() + (size_t)r0 * W : nullptr,
                                     out32 ? nullptr : outw.data() + (size_t)r0 * W, nullptr, nullptr, cnt);
        else
            rc = sgpu_stack_rows(ctx, (const float *)buf[slot].data(), N, W, nr, nr * W, &p,
                                 outf.data() + (size_t)r0 * W, nullptr, nullptr, cnt);
        if (reader.joinable()) reader.join();
        if (rc) break;
        r0 = nxt;
        nr = nnr;
        slot ^= 1;
    }
    if (rc) return rc;
    if (out32 && p.output_norm) {
        // norm_to_0_1_range (median_and_mean.c:557-582, called at :1774-1775)
        // on the assembled image, on the device (output_norm.hip)
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
    std::vector<std::string> hist;
    char h[80];
    std::snprintf(h, sizeof h, "Stacking method: %s (siril_amd MI355X engine)",
                  p.method == SGPU_METHOD_MEDIAN ? "median" : "average with rejection");
    hist.push_back(h);
    std::snprintf(h, sizeof h, "Integration of %d images, rejection %d (%g, %g)", N, p.type_of_rejection,
                  p.sig[0], p.sig[1]);
    hist.push_back(h);
    return out32 ? fits_write(out_path, outf.data(), W, H, -32, hist)
                 : fits_write(out_path, outw.data(), W, H, 16, hist);
}
