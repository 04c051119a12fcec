// capi_check.cpp — a C++ caller of the C-ABI through include/plvi_frontend.h
// only (no OpenCV, no HIP headers), the way the INTEGRATION.md shims call it
// from ORBextractor::operator() / Lineextractor::operator() /
// LineMatcher::match.  Usage: capi_check <frame.raw> <w> <h> <out.bin>
// Writes: int32 status words, then the ORB keypoints / descriptors, the
// keylines / LBD descriptors / line functions and a LineMatcher::match of
// the frame's LBD descriptors against themselves reversed; tests/
// test_capi_native.py compares them with the CPU oracle.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "plvi_frontend.h"

int main(int argc, char** argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s frame.raw w h out.bin\n", argv[0]);
        return 2;
    }
    const int w = atoi(argv[2]), h = atoi(argv[3]);
    std::vector<uint8_t> img((size_t)w * h);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(img.data(), 1, img.size(), f) != img.size()) return 3;
    fclose(f);
    std::vector<int32_t> st;

    plvi_orb_params op = {1000, 1.2f, 8, 20, 7, 0};
    plvi_orb_extractor* orb = nullptr;
    st.push_back(plvi_orb_create(&op, 640, 480, 1, 0, &orb));
    if (!orb) return 4;
    const int cap = 8192;
    std::vector<plvi_keypoint> kps(cap);
    std::vector<uint8_t> desc((size_t)cap * 32);
    int n = -7, mono = -7;
    // ORBextractor.cc:1072-1073: empty image -> -1
    st.push_back(plvi_orb_extract(orb, nullptr, 0, 0, 0, 0, 0, kps.data(), desc.data(), cap, &n, &mono));
    st.push_back(plvi_orb_extract(orb, img.data(), 0, h, (size_t)w, 0, 0, kps.data(), desc.data(), cap, &n, &mono));
    // the frame (any size: 752x480 re-plans the 640x480 handle)
    st.push_back(plvi_orb_extract(orb, img.data(), w, h, (size_t)w, 0, 0, kps.data(), desc.data(), cap, &n, &mono));
    int anyErr = -1;
    st.push_back(plvi_orb_errors(orb, nullptr, &anyErr, nullptr));
    st.push_back(anyErr);
    st.push_back(n);
    st.push_back(mono);

    plvi_line_params lp = {200, 0, 0.8f, 2, 2.0f, 0, 0};
    plvi_line_extractor* lx = nullptr;
    st.push_back(plvi_lines_create(&lp, w, h, 1, 0, &lx));
    if (!lx) return 5;
    const int lcap = 4096;
    std::vector<plvi_keyline> kl(lcap);
    std::vector<uint8_t> ldesc((size_t)lcap * 32);
    std::vector<double> fn((size_t)lcap * 3);
    int nl = -7;
    st.push_back(plvi_lines_extract(lx, img.data(), w, h, (size_t)w, kl.data(), ldesc.data(), fn.data(), lcap, &nl));
    st.push_back(plvi_lines_errors(lx, nullptr, &anyErr, nullptr));
    st.push_back(anyErr);
    st.push_back(nl);

    // LineMatcher::match(desc, reversed desc, 0.9, matches_12)
    std::vector<uint8_t> rev((size_t)nl * 32);
    for (int i = 0; i < nl; ++i)
        for (int b = 0; b < 32; ++b) rev[(size_t)i * 32 + b] = ldesc[(size_t)(nl - 1 - i) * 32 + b];
    std::vector<int> m12(nl > 0 ? nl : 1, -1);
    st.push_back(plvi_line_match(ldesc.data(), nl, rev.data(), nl, 0.9f, m12.data()));

    st.push_back(plvi_orb_destroy(orb));
    st.push_back(plvi_lines_destroy(lx));

    FILE* o = fopen(argv[4], "wb");
    if (!o) return 6;
    const int32_t ns = (int32_t)st.size();
    fwrite(&ns, 4, 1, o);
    fwrite(st.data(), 4, st.size(), o);
    fwrite(kps.data(), sizeof(plvi_keypoint), n > 0 ? n : 0, o);
    fwrite(desc.data(), 32, n > 0 ? n : 0, o);
    fwrite(kl.data(), sizeof(plvi_keyline), nl > 0 ? nl : 0, o);
    fwrite(ldesc.data(), 32, nl > 0 ? nl : 0, o);
    fwrite(fn.data(), 24, nl > 0 ? nl : 0, o);
    fwrite(m12.data(), 4, nl > 0 ? nl : 0, o);
    fclose(o);
    return 0;
}
