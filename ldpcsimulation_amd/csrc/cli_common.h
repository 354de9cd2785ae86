// cli_common.h -- host helpers shared by the reference-compatible CLIs.
#pragma once
#include <fstream>
#include <iterator>
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
