// cli_minsum.cpp -- reference-compatible front-end of the MI355X decoder.
//
// Drop-in for the decodeMinSum family of ereiss123/LDPCsimulation
// (C_implementations/src/decodeMinSum.cpp:72-334) and, built with
// -D beliefPropagation, for decodeBP (src/decodeBP.cpp:58-277: the tanh rule,
// LLR front-end 4y/N0, stop rule 200 errors / 20|10|5 word errors, its own
// parameter block and log line): the same positional CLI
//   decodeMinSum alist R SNR T [Ymax] [Q] [alpha] [delta] logfilename [codewordfile]
// with the variant fixed at compile time by the same -D macros
// (quantizeSamples, saturateSamples, normalizedMS, offsetMS; Makefile:58-65),
// the same stdout (parameters, "Ferr with k errors.", "Incremental result"
// every 5 frames with the error-weight histogram, "Final result") and the
// same appended tab-separated log line (:313-329). The stop rule (:189) is
// applied frame by frame in frame order, so batching never changes the
// statistics.
//
// The decode runs on the GPU through the C ABI (include/ldpc_hip.h). GPU
// options come from the environment so the positional CLI stays identical:
//   LDPC_RNG       glibc (default): the reference's noise -- srandom(seed) +
//                  rand.h rann() on the host, fp64 decode on the GPU; the
//                  output then equals the reference's for the same seed.
//                  philox: counter-based noise generated on the GPU.
//   LDPC_SEED      noise seed (default time(0), as ran_seed(time(0)) :187)
//   LDPC_PRECISION f64 (default: the reference's double) | f32 (opt-in)
//   LDPC_BATCH     frames per GPU launch (default 512 glibc / 65536 philox)
//   LDPC_DEVICE    HIP device index (default 0)
//   LDPC_DRY_RUN   print these settings to stderr and exit before any device call
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "ldpc_hip.h"
#include "cli_common.h"

using std::cout;
using std::endl;

namespace {

// The reference's noise source (inc/rand.h:10-11,19-20): glibc random()
// scaled to [0,1) and a Box-Muller cosine branch whose angle uniform is
// drawn first.
inline double ranf_glibc() { return (double)random() / (1.0 + (double)0x7fffffff); }
inline double rann_glibc()
{
    const double ua = ranf_glibc();
    const double ur = ranf_glibc();
    return std::cos(2.0 * 3.141592654 * ua) * std::sqrt(-2.0 * std::log(1.0 - ur));
}

const char *env_or(const char *k, const char *d)
{
    const char *v = std::getenv(k);
    return (v && *v) ? v : d;
}

[[noreturn]] void die(const char *what)
{
    std::cerr << "ldpc: " << what << ": " << ldpc_last_error() << endl;
    std::exit(1);
}

void print_histogram(const std::vector<long> &h)   // printHistogram (:373-380)
{
    for (size_t i = 0; i < h.size(); ++i)
        if (h[i] > 0) cout << i + 1 << ":\t" << h[i] << endl;
}

// Read "N M / maxdv maxdc" as declared in the alist header (dv, dc of :150-151).

}  // namespace

int main(int argc, char *argv[])
{
    std::vector<std::string> args = {"alist", "R", "SNR", "T"};
#if defined(quantizeSamples) || defined(saturateSamples)
    args.push_back("Ymax");
#endif
#ifdef quantizeSamples
    args.push_back("Q");
#endif
#ifdef normalizedMS
    args.push_back("alpha");
#endif
#ifdef offsetMS
    args.push_back("delta");
#endif
    args.push_back("logfilename");
    args.push_back("[codeword filename]");
#ifdef beliefPropagation
    args = {"alist", "R", "SNR", "T", "logfilename", "[codeword filename]"};   // decodeBP.cpp:60-67
#endif
    if ((size_t)argc != args.size() && (size_t)argc != args.size() + 1) {   // :95-102
        cout << "Usage: " << argv[0];
        for (const auto &a : args) cout << " " << a;
        cout << "\n";
        return 0;
    }

    ldpc_decoder_cfg cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.variant = LDPC_MS;
#ifdef beliefPropagation
    cfg.variant = LDPC_BP;
#endif
    int idx = 1;
    ldpc_graph *H = nullptr;
    if (ldpc_graph_load_alist(argv[idx++], &H) != LDPC_OK) die("loading alist");
    int N = 0, M = 0;
    ldpc_graph_info(H, &N, &M, nullptr, nullptr, nullptr);
    cout << "PARAMETERS: \n alist = \t" << argv[1] << endl;
    const double R = std::atof(argv[idx++]);
    cout << " R = \t" << R << endl;
    const double SNR = std::atof(argv[idx++]);
    cout << " SNR = \t" << SNR << endl;
    const int T = std::atoi(argv[idx++]);
    cout << " T = \t" << T << endl;
    cfg.T = T;
#ifdef saturateSamples
    const double Ymax = std::atof(argv[idx++]);
    cout << "Applying sample clipping with Ymax = +/-" << Ymax << endl;
    cfg.saturate = 1;
    cfg.ymax = Ymax;
#endif
#ifdef quantizeSamples
    const double Ymax = std::atof(argv[idx++]);
    const int Q = std::atoi(argv[idx++]);
    const double Nq = std::pow(2.0, Q);
    cout << "Applying sample quantization with Ymax = +/-" << Ymax << " on " << Q << " bits with " << Nq - 1
         << " non-zero levels." << endl;
    cfg.quantize = 1;
    cfg.ymax = Ymax;
    cfg.qbits = Q;
#endif
#ifdef normalizedMS
    const double alpha = std::atof(argv[idx++]);
    cout << "Using normalization with alpha=" << alpha << endl;
    cfg.variant = LDPC_NMS;
    cfg.alpha = alpha;
#endif
#ifdef offsetMS
    const double delta = std::atof(argv[idx++]);
    cout << "Using offset MS with delta=" << delta << endl;
    cfg.variant = LDPC_OMS;
    cfg.delta = delta;
#endif
    const std::string logfilename(argv[idx++]);
    cout << " log = \t" << logfilename << endl;

    // Codeword file (:136-143, :193-212): lines of '0'/'1', cycled in order.
    std::vector<std::string> cw_lines;
    const bool use_cw = (size_t)argc == args.size() + 1;
    if (use_cw) {
        cout << "\nUsing codewords from " << argv[idx] << endl;
        cw_lines = reference_codeword_lines(argv[idx]);
    } else {
        cout << "\nUsing all-zero sequence.\n";
    }

    const double N0 = std::pow(10.0, -SNR / 10.0) / R;   // :146-147
    const double sigma = std::sqrt(N0 / 2.0);
    int dv = 0, dc = 0;
    alist_header(argv[1], dv, dc);
    cout << "Simulating Min-Sum decoding on code with N=" << N << ", M=" << M << ", R=" << R << ", dv=" << dv
         << ", dc=" << dc << endl;
#ifdef beliefPropagation
    cout << "\nParameters are:\n\tSNR\t" << SNR << endl;   // decodeBP.cpp:114
    cfg.n0 = N0;
    const int minWordErrors = N > 50000 ? 5 : (N > 10000 ? 10 : 20);   // decodeBP.cpp:145-147
#else
    cout << "\nParameters are:\n\tSNR\t" << SNR << "\n\tN0\t" << N0 << "\n\tsigma\t" << sigma << endl;
    const int minWordErrors = 40;   // :189
#endif

    // ---- GPU setup ----
    const std::string rng = env_or("LDPC_RNG", "glibc");
    const bool philox = rng == "philox";
    if (!philox && rng != "glibc") {
        std::cerr << "ldpc: LDPC_RNG must be glibc or philox" << endl;
        return 1;
    }
    const std::string prec = env_or("LDPC_PRECISION", "f64");
    cfg.precision = prec == "f32" ? LDPC_F32 : LDPC_F64;
    const long long seed = std::atoll(env_or("LDPC_SEED", std::to_string((long long)time(0)).c_str()));
    const int batch = std::atoi(env_or("LDPC_BATCH", philox ? "65536" : "512"));
    const int device = std::atoi(env_or("LDPC_DEVICE", "0"));
    if (batch <= 0) {
        std::cerr << "ldpc: LDPC_BATCH must be > 0" << endl;
        return 1;
    }
    if (std::getenv("LDPC_DRY_RUN")) {   // report the GPU settings and stop before any device call
        std::cerr << "ldpc: rng=" << rng << " precision=" << (cfg.precision == LDPC_F64 ? "f64" : "f32")
                  << " batch=" << batch << " device=" << device << endl;
        return 0;
    }
    ldpc_ctx *ctx = nullptr;
    if (ldpc_ctx_create(device, H, batch, &ctx) != LDPC_OK) die("creating device context");

    // Transmitted codewords per frame (bipolar, :202-211). An invalid symbol
    // is reported and leaves c[i] as it was, like the reference.
    std::vector<int8_t> c_cur(N, 1);
    auto load_codeword = [&](long frame, std::vector<int8_t> &c) {
        apply_codeword_line(cw_lines[(size_t)(frame % (long)cw_lines.size())], N, c, cout);
    };
    if (philox && use_cw) {
        std::vector<uint8_t> bits((size_t)cw_lines.size() * N);
        for (size_t r = 0; r < cw_lines.size(); ++r) {
            load_codeword((long)r, c_cur);
            for (int i = 0; i < N; ++i) bits[r * N + i] = c_cur[i] < 0 ? 1 : 0;
        }
        if (ldpc_sim_set_codewords(ctx, bits.data(), (int)cw_lines.size()) != LDPC_OK) die("uploading codewords");
    }

    long errors = 0, uncodedErrors = 0, totalBits = 0, totalWords = 0, wordErrors = 0, totalIterations = 0;
    std::vector<long> hist(N, 0);
    std::vector<ldpc_frame_result> res(batch);
    std::vector<double> y;
    std::vector<int8_t> cbuf;
    if (!philox) {
        srandom((unsigned)seed);   // ran_seed (:187)
        y.resize((size_t)batch * N);
        if (use_cw) cbuf.resize((size_t)batch * N);
    }
    std::vector<float> yf;
    long generated = 0;
    bool done = false;
    while (!done) {
        if (philox) {
            ldpc_counts tmp{};
            if (ldpc_sim_batch(ctx, SNR, R, &cfg, (uint64_t)seed, 0u, (uint64_t)generated, batch, res.data(), &tmp) !=
                LDPC_OK)
                die("simulating batch");
        } else {
            for (int f = 0; f < batch; ++f) {   // AWGN exactly as :214-216, frame order
                if (use_cw) load_codeword(generated + f, c_cur);
                double *yr = y.data() + (size_t)f * N;
                for (int i = 0; i < N; ++i) yr[i] = (double)c_cur[i] * (1.0 + sigma * rann_glibc());
                if (use_cw) std::memcpy(cbuf.data() + (size_t)f * N, c_cur.data(), (size_t)N);
            }
            const void *yin = y.data();
            if (cfg.precision == LDPC_F32) {
                yf.assign(y.begin(), y.end());
                yin = yf.data();
            }
            if (ldpc_decode_batch(ctx, yin, batch, &cfg, use_cw ? cbuf.data() : nullptr, nullptr, res.data(),
                                  nullptr) != LDPC_OK)
                die("decoding batch");
        }
        generated += batch;
        for (int f = 0; f < batch; ++f) {
            if (!(errors < 200 || wordErrors < minWordErrors)) {   // :189
                done = true;
                break;
            }
            const int newErrors = res[f].bit_err;
            uncodedErrors += res[f].uncoded_bit_err;
            if (newErrors > 0) {   // :272-283
                cout << "Ferr with " << newErrors << " errors.";
                cout << endl;
                errors += newErrors;
                hist[newErrors - 1]++;
                wordErrors++;
            }
            totalWords++;   // :286-288
            totalBits += N;
            totalIterations += T;
            if ((totalWords % 5) == 0) {   // :292-298
                cout << "\nIncremental result: " << errors << " bit errs in " << totalWords
                     << " words, BER=" << (double)errors / totalBits
                     << ". Average iterations = " << (double)totalIterations / totalWords
                     << ". Word error=" << wordErrors << ". Uncoded errors = " << uncodedErrors
                     << ", uncBER=" << (double)uncodedErrors / totalBits << "\nError weights:\n";
                print_histogram(hist);
            }
        }
    }

    cout << "\nFinal result: " << errors << " bit errs in " << totalWords << " words, BER=" << (double)errors / totalBits
         << ". Average iterations = " << (double)totalIterations / totalWords << ". Uncoded errors = " << uncodedErrors
         << ", uncBER=" << (double)uncodedErrors / totalBits << endl;

    std::ofstream of(logfilename.c_str(), std::ios::app);   // :313-329
    const char tab = '\t';
    of << SNR << tab << (double)errors / totalBits << tab << (double)totalIterations / totalWords << tab
       << (double)wordErrors / totalWords << tab << T << tab;
#if defined(saturateSamples) || defined(quantizeSamples)
    of << Ymax << tab;
#endif
#ifdef normalizedMS
    of << alpha << tab;
#endif
#ifdef offsetMS
    of << delta << tab;
#endif
    of << argv[1] << endl;
    of.close();

    ldpc_ctx_destroy(ctx);
    ldpc_graph_destroy(H);
    return 0;
}
