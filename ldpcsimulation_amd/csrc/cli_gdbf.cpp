// cli_gdbf.cpp -- reference-compatible front-end of the MI355X GDBF / NGDBF
// bit-flipping decoders.
//
// Drop-in for the decodeGDBF family of ereiss123/LDPCsimulation
// (C_implementations/src/decodeGDBF.cpp:86-454) in its parallel-flip mode:
// the same positional CLI
//   decodeXGDBF alist R SNR T theta logfilename [noiseScale] [NQ] [lambda]
//               [alpha] [windowsize] [Ymax] [codewordfile]
// with the variant fixed at compile time by the same -D macros (addNoise,
// quantizeSamples, thresholdAdaptation, weightSyndromes, outputSmoothing,
// saturateSamples; Makefile:33-53), the same stdout (parameters, "Ferr with k
// errors." [+ " All checks satisfied."], "Incremental result" every
// round(100e3/N) frames with the histogram, "Final result") and the same
// appended log line (:425-452). Stop rule: errors >= 200 and word errors >=
// 20 (10 for N > 10000, 5 for N > 50000), frame by frame (:221-226).
//
// Environment (the positional CLI stays identical):
//   LDPC_RNG       glibc (default): the reference's noise -- glibc random()
//                  TYPE_3 seeded like ran_seed(seed) and rand.h rann(), drawn
//                  on the host in the reference's order (channel, then one
//                  row of N perturbations per iteration that passes its
//                  syndrome check); frames are decoded one at a time in fp64
//                  on the GPU, so the output equals the reference's.
//                  philox: channel and perturbations generated on the GPU,
//                  batched (LDPC_BATCH frames per launch).
//   LDPC_SEED, LDPC_PRECISION, LDPC_BATCH, LDPC_DEVICE, LDPC_DRY_RUN as cli_minsum.cpp.
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

// glibc random()/srandom() TYPE_3 (x^31 + x^3 + 1 additive feedback), kept
// in a copyable object so a frame's perturbation rows can be drawn ahead and
// the stream then advanced by exactly the rows the decoder used.
struct GlibcRandom {
    int32_t r[31];
    int f = 3, b = 0;
    explicit GlibcRandom(uint32_t seed)
    {
        int32_t w = (int32_t)(seed ? seed : 1u);
        r[0] = w;
        for (int i = 1; i < 31; ++i) {   // 16807 * w mod (2^31 - 1), Schrage
            const int32_t hi = w / 127773, lo = w % 127773;
            w = 16807 * lo - 2836 * hi;
            if (w < 0) w += 2147483647;
            r[i] = w;
        }
        for (int i = 0; i < 310; ++i) next();
    }
    int32_t next()
    {
        const uint32_t v = (uint32_t)r[f] + (uint32_t)r[b];
        r[f] = (int32_t)v;
        if (++f == 31) f = 0;
        if (++b == 31) b = 0;
        return (int32_t)(v >> 1);
    }
    double ranf() { return (double)next() / (1.0 + (double)0x7fffffff); }   // rand.h:10-11
    double ranu() { return (1.0 + (double)next()) / (2.0 + (double)0x7fffffff); }   // rand.h:13-14
    double rann()                                                            // rand.h:19-20
    {
        const double ua = ranf();
        const double ur = ranf();
        return std::cos(2.0 * 3.141592654 * ua) * std::sqrt(-2.0 * std::log(1.0 - ur));
    }
};

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

void print_histogram(const std::vector<int> &h)   // printHistogram (:465-472)
{
    for (size_t i = 0; i < h.size(); ++i)
        if (h[i] > 0) cout << i + 1 << ":\t" << h[i] << endl;
}


}  // namespace

int main(int argc, char *argv[])
{
    std::vector<std::string> args = {"alist", "R", "SNR", "T", "theta", "logfilename"};   // :88-113
#if defined(addNoise) || defined(quantizeProbabilities)
    args.push_back("noiseScale");
#endif
#ifdef quantizeSamples
    args.push_back("NQ");
#endif
#ifdef thresholdAdaptation
    args.push_back("lambda");
#endif
#ifdef weightSyndromes
    args.push_back("alpha");
#endif
#ifdef outputSmoothing
    args.push_back("windowsize");
#endif
#ifdef saturateSamples
    args.push_back("Ymax");
#endif
    args.push_back("[codeword filename]");
    if ((size_t)argc != args.size() && (size_t)argc != args.size() + 1) {   // :116-123
        cout << "Usage: " << argv[0];
        for (const auto &a : args) cout << " " << a;
        cout << "\n";
        return 0;
    }

    ldpc_gdbf_cfg cfg;
    std::memset(&cfg, 0, sizeof cfg);
    // the reference's defaults (:48-56)
    cfg.lambda = 0.991;
    cfg.alpha = 2.25;
    cfg.ymax = 2.25;
    cfg.windowsize = 64;
    cfg.noise_scale = 1.0;
    cfg.nq = 16;
    int idx = 1;
    ldpc_graph *H = nullptr;
    if (ldpc_graph_load_alist(argv[idx++], &H) != LDPC_OK) die("loading alist");
    int N = 0, M = 0;
    ldpc_graph_info(H, &N, &M, nullptr, nullptr, nullptr);
    cout << "PARAMETERS: \n alist = \t" << argv[1] << endl;   // :128-163
    const double R = std::atof(argv[idx++]);
    cout << " R = \t" << R << endl;
    const double SNR = std::atof(argv[idx++]);
    cout << " SNR = \t" << SNR << endl;
    const int T = std::atoi(argv[idx++]);
    cout << " T = \t" << T << endl;
    cfg.T = T;
    const double theta = std::atof(argv[idx++]);
    cout << " theta = \t" << theta << endl;
    cfg.theta = theta;
    const std::string logfilename(argv[idx++]);
    cout << " log = \t" << logfilename << endl;
#if defined(addNoise) || defined(quantizeProbabilities)
    cfg.noise_scale = std::atof(argv[idx++]);
    cout << " noiseScale = \t" << cfg.noise_scale << endl;
#endif
#ifdef addNoise
    cfg.flags |= LDPC_GDBF_NOISE;
#endif
#ifdef quantizeProbabilities
    cfg.flags |= LDPC_GDBF_QPROB;   // :562-597
#endif
#ifdef sequentialmode
    cfg.flags |= LDPC_GDBF_SEQUENTIAL;   // :285-289
#endif
#ifdef modeswitching
    cfg.flags |= LDPC_GDBF_MODESWITCH;   // :309-345, Tswitch = 0 (:51)
#endif
#ifdef quantizeSamples
    cfg.flags |= LDPC_GDBF_QUANTIZE;
    cfg.nq = std::atoi(argv[idx++]);
    cout << " NQ = \t" << cfg.nq << endl;
#endif
#ifdef thresholdAdaptation
    cfg.flags |= LDPC_GDBF_ADAPT;
    cfg.lambda = std::atof(argv[idx++]);
    cout << " lambda = \t" << cfg.lambda << endl;
#endif
#ifdef weightSyndromes
    cfg.flags |= LDPC_GDBF_WEIGHT;
    cfg.alpha = std::atof(argv[idx++]);
    cout << " alpha = \t" << cfg.alpha << endl;
#endif
#ifdef outputSmoothing
    cfg.flags |= LDPC_GDBF_SMOOTH;
    cfg.windowsize = std::atoi(argv[idx++]);
    cout << "windowsize = \t" << cfg.windowsize << endl;
#endif
#ifdef saturateSamples
    cfg.flags |= LDPC_GDBF_SATURATE;
    cfg.ymax = std::atof(argv[idx++]);
    cout << " Ymax = \t" << cfg.ymax << endl;
#endif

    std::vector<std::string> cw_lines;   // :165-172, :230-249
    const bool use_cw = (size_t)argc == args.size() + 1;
    if (use_cw) {
        cout << "\nUsing codewords from " << argv[idx] << endl;
        cw_lines = reference_codeword_lines(argv[idx]);
    } else {
        cout << "\nUsing all-zero sequence.\n";
    }

    const double N0 = std::pow(10.0, -SNR / 10.0) / R;   // :175-176
    const double sigma = std::sqrt(N0 / 2.0);
    int dv = 0, dc = 0;
    alist_header(argv[1], dv, dc);
    cout << "Simulating GDBF decoding on code with N=" << N << ", M=" << M << ", R=" << R << ", dv=" << dv
         << ", dc=" << dc << endl;
    cout << "\nParameters are:\n\tSNR\t" << SNR << "\n\tN0\t" << N0 << "\n\tsigma\t" << sigma << endl;

    // ---- GPU setup ----
    const std::string rng = env_or("LDPC_RNG", "glibc");
    const bool philox = rng == "philox";
    if (!philox && rng != "glibc") {
        std::cerr << "ldpc: LDPC_RNG must be glibc or philox" << endl;
        return 1;
    }
    const std::string prec = env_or("LDPC_PRECISION", "f64");   // the reference's double; f32 opt-in
    cfg.precision = prec == "f32" ? LDPC_F32 : LDPC_F64;
    const long long seed = std::atoll(env_or("LDPC_SEED", std::to_string((long long)time(0)).c_str()));
    const int batch = philox ? std::atoi(env_or("LDPC_BATCH", "65536")) : 1;
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

    int minWordErrors = 20;   // :221-223
    if (N > 10000) minWordErrors = 10;
    if (N > 50000) minWordErrors = 5;
    const int reportInterval = (int)std::round(100e3 / N);   // :403
    long errors = 0, uncodedErrors = 0, totalBits = 0, totalWords = 0, wordErrors = 0, totalIterations = 0;
    long smoothingUsed = 0;
    std::vector<int> hist(N, 0);
    std::vector<ldpc_frame_result> res(batch);
    GlibcRandom g((uint32_t)seed);   // ran_seed(time(0)) (:224)
    std::vector<double> y, pert;
    std::vector<float> yf, pf;
    const bool noise = (cfg.flags & LDPC_GDBF_NOISE) != 0;
    const bool qprob = (cfg.flags & LDPC_GDBF_QPROB) != 0;   // ranu() per bit and iteration (:588)
    const double noiseSigma = sigma * cfg.noise_scale;   // :296
    if (!philox) {
        y.resize(N);
        if (noise || qprob) pert.resize((size_t)N * (T > 0 ? T : 1));
    }
    long generated = 0;
    bool done = false;
    while (!done) {
        if (philox) {
            ldpc_counts tmp{};
            if (ldpc_gdbf_sim_batch(ctx, SNR, R, &cfg, (uint64_t)seed, 0u, (uint64_t)generated, batch, res.data(),
                                    &tmp) != LDPC_OK)
                die("simulating batch");
        } else {
            if (use_cw) load_codeword(generated, c_cur);
            for (int i = 0; i < N; ++i) y[i] = (double)c_cur[i] * (1.0 + sigma * g.rann());   // :251-253
            if (noise) {   // the rows this frame may use, drawn ahead from a copy
                GlibcRandom ahead = g;
                for (size_t k = 0; k < pert.size(); ++k) pert[k] = noiseSigma * ahead.rann();
            }
            if (qprob) {
                GlibcRandom ahead = g;
                for (size_t k = 0; k < pert.size(); ++k) pert[k] = ahead.ranu();
                cfg.qsigma = noiseSigma;   // symNodeUpdates' sigma (:296, :353)
            }
            const void *yin = y.data(), *pin = (noise || qprob) ? pert.data() : nullptr;
            if (cfg.precision == LDPC_F32) {
                yf.assign(y.begin(), y.end());
                pf.assign(pert.begin(), pert.end());
                yin = yf.data();
                pin = (noise || qprob) ? pf.data() : nullptr;
            }
            if (ldpc_gdbf_decode_batch(ctx, yin, pin, 1, &cfg, use_cw ? c_cur.data() : nullptr, nullptr, res.data(),
                                       nullptr) != LDPC_OK)
                die("decoding frame");
            if (noise)   // advance by the rows the decoder drew (one per iteration run, :318-333)
                for (long k = 0; k < (long)N * res[0].iters; ++k) (void)g.rann();
            if (qprob)
                for (long k = 0; k < (long)N * res[0].iters; ++k) (void)g.ranu();
        }
        generated += batch;
        for (int f = 0; f < batch; ++f) {
            if (!((errors < 200) || (wordErrors < minWordErrors))) {   // :226
                done = true;
                break;
            }
            const int it = res[f].iters;
            const bool satisfied = it < T;
            if ((cfg.flags & LDPC_GDBF_SMOOTH) && it > T - cfg.windowsize) smoothingUsed++;   // :371-375
            const int newErrors = res[f].bit_err;
            uncodedErrors += res[f].uncoded_bit_err;
            if (newErrors > 0) {   // :380-394
                cout << "Ferr with " << newErrors << " errors.";
                if (satisfied)
                    cout << " All checks satisfied.\n";
                else
                    cout << endl;
                errors += newErrors;
                hist[newErrors - 1]++;
                wordErrors++;
            }
            totalWords++;   // :397-399
            totalBits += N;
            totalIterations += it;
            if ((totalWords % reportInterval) == 0) {   // :403-410
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

    std::ofstream of(logfilename.c_str(), std::ios::app);   // :425-452
    const char tab = '\t';
    of << SNR << tab << (double)errors / totalBits << tab << (double)totalIterations / totalWords << tab
       << (double)wordErrors / totalWords << tab << totalBits << tab << totalWords << tab << T << tab << theta << tab;
#if defined(addNoise) || defined(quantizeProbabilities)
    of << cfg.noise_scale << tab;
#endif
#ifdef quantizeSamples
    of << cfg.nq << tab;
#endif
#ifdef thresholdAdaptation
    of << cfg.lambda << tab;
#endif
#ifdef weightSyndromes
    of << cfg.alpha << tab;
#endif
#ifdef outputSmoothing
    of << smoothingUsed << tab << (double)smoothingUsed / totalWords << tab;
    of << cfg.windowsize << tab;
#endif
#ifdef saturateSamples
    of << cfg.ymax << tab;
#endif
    of << argv[1] << endl;
    of.close();

    ldpc_ctx_destroy(ctx);
    ldpc_graph_destroy(H);
    return 0;
}
