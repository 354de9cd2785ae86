// cli_common.h -- host helpers shared by the reference-compatible CLIs.
#pragma once
#include <cstdint>
#include <fstream>
#include <iterator>
#include <ostream>
#include <string>
#include <vector>

// The codeword lines the reference's frame loop cycles through
// (decodeMinSum.cpp:193-200, decodeGDBF.cpp:230-237): each frame does
// getline(); when that sets eof() the file is rewound and the first line read
// instead. A last line without a trailing '\n' therefore sets eof() as it is
// read and is never used (unless it is the only line); a file that ends with
// '\n' cycles through all its lines; an empty file yields one empty line
// (every symbol invalid).
inline std::vector<std::string> reference_codeword_lines(const char *path)
{
    std::ifstream f(path, std::ios::binary);
    const std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<std::string> lines;
    size_t at = 0;
    while (at < text.size()) {
        const size_t nl = text.find('\n', at);
        if (nl == std::string::npos) {
            lines.push_back(text.substr(at));   // unterminated last line
            if (lines.size() > 1) lines.pop_back();
            break;
        }
        lines.push_back(text.substr(at, nl - at));
        at = nl + 1;
    }
    if (lines.empty()) lines.push_back(std::string());
    return lines;
}

// One codeword line into the bipolar transmitted word c[0..N) (decodeMinSum.cpp:202-211,
// decodeGDBF.cpp:239-248): '1' -> -1, '0' -> +1; any other symbol, or a line shorter
// than N, is reported on `log` and leaves c[i] as it was, as in the reference.
inline void apply_codeword_line(const std::string &s, int N, std::vector<int8_t> &c, std::ostream &log)
{
    if ((int)c.size() < N) c.resize(N, 1);
    for (int i = 0; i < N; ++i) {
        const char ch = i < (int)s.size() ? s[i] : '\0';
        if (ch == '1') c[i] = -1;
        else if (ch == '0') c[i] = +1;
        else log << "Got an invalid symbol at index " << i << std::endl;
    }
}

// "N M / maxdv maxdc" as the alist header declares them (the dv, dc the reference
// prints, decodeMinSum.cpp:150-151); a field that cannot be read is 0.
inline void alist_header(const char *path, int &dv, int &dc)
{
    std::ifstream f(path);
    int n = 0, m = 0;
    dv = dc = 0;
    f >> n >> m >> dv >> dc;
}
