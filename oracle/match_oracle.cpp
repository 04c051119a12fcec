// oracle/match_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the Hamming matchers on the path ("parity unpinned":
// no reference test pins them; restated from the cited lines):
//   DescriptorDistance  src/ORBmatcher.cc:2350-2366 (SWAR popcount, >>24)
//   LineMatcher::DescriptorDistance src/LineMatcher.cpp:487-499 (>>25 quirk)
//   BFMatcher::knnMatch(k=2)  OpenCV 4.2 batchDistance K-insertion
//   LineMatcher::matchNNR / match  src/LineMatcher.cpp:41-111
#include <climits>
#include <cstdint>
#include <cstring>
#include <vector>

static int descriptor_distance(const uint8_t* a, const uint8_t* b, int shift) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        int32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        unsigned int v = (unsigned)(pa ^ pb);
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> shift);
    }
    return dist;
}

extern "C" int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b, 24); }
extern "C" int oracle_line_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    return descriptor_distance(a, b, 25);
}

extern "C" void oracle_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int* i0, int* d0, int* i1, int* d1) {
    const int K = 2;
    for (int i = 0; i < nq; ++i) {
        int dist[K] = {INT_MAX, INT_MAX}, nidx[K] = {-1, -1};
        for (int j = 0; j < nt; ++j) {
            int d = descriptor_distance(q + (size_t)i * 32, t + (size_t)j * 32, 24);
            if (d < dist[K - 1]) {
                int k;
                for (k = K - 2; k >= 0 && dist[k] > d; k--) {
                    nidx[k + 1] = nidx[k];
                    dist[k + 1] = dist[k];
                }
                nidx[k + 1] = j;
                dist[k + 1] = d;
            }
        }
        i0[i] = nidx[0]; d0[i] = dist[0]; i1[i] = nidx[1]; d1[i] = dist[1];
    }
}

extern "C" int oracle_match_nnr(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, int* m12) {
    std::vector<int> i0(n1), a(n1), i1(n1), b(n1);
    oracle_knn2(d1, n1, d2, n2, i0.data(), a.data(), i1.data(), b.data());
    int matches = 0;
    for (int idx = 0; idx < n1; ++idx) {
        m12[idx] = -1;
        if ((float)a[idx] < (float)b[idx] * nnr) {
            m12[idx] = i0[idx];
            ++matches;
        }
    }
    return matches;
}

extern "C" int oracle_match(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, int* m12) {
    std::vector<int> m21(n2 > 0 ? n2 : 1);
    int matches = oracle_match_nnr(d1, n1, d2, n2, nnr, m12);
    oracle_match_nnr(d2, n2, d1, n1, nnr, m21.data());
    for (int i1 = 0; i1 < n1; ++i1) {
        int& i2 = m12[i1];
        if (i2 >= 0 && m21[i2] != i1) {
            i2 = -1;
            --matches;
        }
    }
    return matches;
}
