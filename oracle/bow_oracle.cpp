// oracle/bow_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of DBoW2's vocabulary path used by Frame::ComputeBoW
// (src/Frame.cc:1115-1122) and KeyFrame::ComputeBoW (src/KeyFrame.cc:111):
//   TemplatedVocabulary::loadFromTextFile  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424
//   TemplatedVocabulary::transform(feature, word, weight, nid, levelsup)  :1217-1259
//   TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)  :1126-1194
//   BowVector::addWeight / addIfNotExist / normalize  BowVector.cpp:34-84
//   FeatureVector::addFeature  FeatureVector.cpp:31-45
//   FORB::distance / fromString  FORB.cpp:81-101, 120-135
//   scoring -> (mustNormalize, norm)  ScoringObject.h:74-89
// "Parity unpinned": the reference ships no tests and its vocabulary blob
// (Vocabulary/ORBvoc.txt) is absent; this follows the cited lines with
// std::map containers and iostream parsing exactly like the reference.
//
// The loader's `while(!f.eof()) getline` loop reads one more (empty) line
// after the file's final newline and creates one more node from it.  On that
// empty stream `ssnode >> pid` fails in the istream sentry, so pid and
// nIsLeaf keep whatever the uninitialised locals held and the descriptor
// bytes stay uninitialised (FORB::fromString): the node is undefined
// behaviour in the reference.  Default (emulate_tail = 0): no such node.
// emulate_tail != 0 models one outcome -- pid and nIsLeaf reading 0, i.e. a
// weight-0, zero-descriptor, non-word child of the root -- unpinned.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Node {
    unsigned id = 0, parent = 0, word_id = 0;
    double weight = 0;
    std::vector<unsigned> children;
    uint8_t desc[32] = {0};
    bool isLeaf() const { return children.empty(); }
};

struct Vocab {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<Node> nodes;
    std::vector<unsigned> words;  // word id -> node id
};

int forb_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        int32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        unsigned int v = (unsigned)(pa ^ pb);
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

// single-feature descent (TemplatedVocabulary.h:1217-1259)
void transform1(const Vocab& V, const uint8_t* f, unsigned& word_id, double& weight, unsigned* nid, int levelsup) {
    const int nid_level = V.L - levelsup;
    if (nid_level <= 0 && nid != nullptr) *nid = 0;
    unsigned final_id = 0;
    int current_level = 0;
    do {
        ++current_level;
        const std::vector<unsigned> nodes = V.nodes[final_id].children;
        final_id = nodes[0];
        double best_d = forb_distance(f, V.nodes[final_id].desc);
        for (size_t j = 1; j < nodes.size(); ++j) {
            const unsigned id = nodes[j];
            const double d = forb_distance(f, V.nodes[id].desc);
            if (d < best_d) {
                best_d = d;
                final_id = id;
            }
        }
        if (nid != nullptr && current_level == nid_level) *nid = final_id;
    } while (!V.nodes[final_id].isLeaf());
    word_id = V.nodes[final_id].word_id;
    weight = V.nodes[final_id].weight;
}

void must_normalize(int scoring, bool& must, int& norm) {
    // ScoringObject.h:74-89: L1, L2, ChiSquare, KL, Bhattacharyya normalise
    // (L2 only for L2_NORM); DotProduct does not.
    must = scoring != 5;
    norm = scoring == 1 ? 2 : 1;
}

}  // namespace

extern "C" void* oracle_vocab_load(const char* path, int emulate_tail) {
    std::ifstream f(path);
    if (!f.is_open() || f.eof()) return nullptr;
    auto* V = new Vocab;
    std::string s;
    std::getline(f, s);
    std::stringstream ss;
    ss << s;
    int n1 = 0, n2 = 0;
    ss >> V->k >> V->L >> n1 >> n2;
    if (V->k < 0 || V->k > 20 || V->L < 1 || V->L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
        delete V;
        return nullptr;
    }
    V->scoring = n1;
    V->weighting = n2;
    V->nodes.resize(1);
    V->nodes[0].id = 0;
    while (!f.eof()) {
        std::string snode;
        std::getline(f, snode);
        if (snode.empty() && f.eof() && !emulate_tail) break;
        std::stringstream ssnode;
        ssnode << snode;
        const unsigned nid = (unsigned)V->nodes.size();
        V->nodes.resize(V->nodes.size() + 1);
        V->nodes[nid].id = nid;
        int pid = 0;
        ssnode >> pid;
        if (pid < 0 || (unsigned)pid >= nid) {
            delete V;
            return nullptr;
        }
        V->nodes[nid].parent = (unsigned)pid;
        V->nodes[pid].children.push_back(nid);
        int nIsLeaf = 0;
        ssnode >> nIsLeaf;
        std::stringstream ssd;
        for (int i = 0; i < 32; ++i) {
            std::string e;
            ssnode >> e;
            ssd << e << " ";
        }
        {  // FORB::fromString
            std::stringstream sd(ssd.str());
            for (int i = 0; i < 32; ++i) {
                int n;
                sd >> n;
                if (!sd.fail()) V->nodes[nid].desc[i] = (unsigned char)n;
            }
        }
        ssnode >> V->nodes[nid].weight;
        if (nIsLeaf > 0) {
            V->nodes[nid].word_id = (unsigned)V->words.size();
            V->words.push_back(nid);
        }
    }
    return V;
}

// Build from arrays (node i+1 = row i, file order): the same structure the
// text loader produces, for large synthetic vocabularies.
extern "C" void* oracle_vocab_create(int k, int L, int scoring, int weighting, int n, const int* parent,
                                     const uint8_t* is_leaf, const uint8_t* desc, const double* weight) {
    auto* V = new Vocab;
    V->k = k; V->L = L; V->scoring = scoring; V->weighting = weighting;
    V->nodes.resize(1);
    for (int i = 0; i < n; ++i) {
        const unsigned nid = (unsigned)V->nodes.size();
        V->nodes.resize(nid + 1);
        Node& d = V->nodes[nid];
        d.id = nid;
        d.parent = (unsigned)parent[i];
        V->nodes[parent[i]].children.push_back(nid);
        std::memcpy(d.desc, desc + (size_t)32 * i, 32);
        d.weight = weight[i];
        if (is_leaf[i]) {
            d.word_id = (unsigned)V->words.size();
            V->words.push_back(nid);
        }
    }
    return V;
}

extern "C" void oracle_vocab_free(void* h) { delete static_cast<Vocab*>(h); }

extern "C" void oracle_vocab_info(void* h, int* info) {
    const Vocab& V = *static_cast<Vocab*>(h);
    info[0] = V.k; info[1] = V.L; info[2] = V.scoring; info[3] = V.weighting;
    info[4] = (int)V.nodes.size(); info[5] = (int)V.words.size();
}

// Node table dump (node 0 = root): parent, first/num children, word id, weight, descriptor.
extern "C" void oracle_vocab_nodes(void* h, int* parent, int* nchild, unsigned* word, double* weight, uint8_t* desc,
                                   int* children) {
    const Vocab& V = *static_cast<Vocab*>(h);
    int c = 0;
    for (size_t i = 0; i < V.nodes.size(); ++i) {
        parent[i] = (int)V.nodes[i].parent;
        nchild[i] = (int)V.nodes[i].children.size();
        word[i] = V.nodes[i].word_id;
        weight[i] = V.nodes[i].weight;
        std::memcpy(desc + 32 * i, V.nodes[i].desc, 32);
        for (unsigned ch : V.nodes[i].children) children[c++] = (int)ch;
    }
}

// transform(features, BowVector&, FeatureVector&, levelsup)
// (TemplatedVocabulary.h:1126-1194).  Outputs: BowVector as (word, value)
// in map order; FeatureVector as CSR (node, off, idx) in map order; per
// feature word / weight / nid of the descent.  Returns 0.
extern "C" int oracle_vocab_transform(void* h, const uint8_t* desc, int n, int levelsup, unsigned* bow_word,
                                      double* bow_value, int* bow_n, unsigned* fv_node, int* fv_off, unsigned* fv_idx,
                                      int* fv_n, unsigned* feat_word, double* feat_w, unsigned* feat_nid) {
    const Vocab& V = *static_cast<Vocab*>(h);
    std::map<unsigned, double> v;
    std::map<unsigned, std::vector<unsigned>> fv;
    *bow_n = 0;
    *fv_n = 0;
    fv_off[0] = 0;
    if (V.words.empty()) return 0;
    bool must;
    int norm;
    must_normalize(V.scoring, must, norm);
    const bool tf = V.weighting == 0 || V.weighting == 1;
    for (int i = 0; i < n; ++i) {
        unsigned id = 0, nid = 0;
        double w = 0;
        transform1(V, desc + (size_t)32 * i, id, w, &nid, levelsup);
        if (feat_word) feat_word[i] = id;
        if (feat_w) feat_w[i] = w;
        if (feat_nid) feat_nid[i] = nid;
        if (w > 0) {
            auto vit = v.lower_bound(id);
            if (tf) {
                if (vit != v.end() && !(id < vit->first)) vit->second += w;  // addWeight
                else v.insert(vit, {id, w});
            } else {
                if (vit == v.end() || id < vit->first) v.insert(vit, {id, w});  // addIfNotExist
            }
            auto fit = fv.lower_bound(nid);  // addFeature
            if (fit != fv.end() && fit->first == nid) fit->second.push_back((unsigned)i);
            else fit = fv.insert(fit, {nid, std::vector<unsigned>()}), fit->second.push_back((unsigned)i);
        }
    }
    if (tf && !v.empty() && !must) {
        const double nd = (double)v.size();
        for (auto& e : v) e.second /= nd;
    }
    if (must) {  // BowVector::normalize
        double nrm = 0.0;
        if (norm == 1) {
            for (auto& e : v) nrm += std::fabs(e.second);
        } else {
            for (auto& e : v) nrm += e.second * e.second;
            nrm = std::sqrt(nrm);
        }
        if (nrm > 0.0)
            for (auto& e : v) e.second /= nrm;
    }
    int j = 0;
    for (auto& e : v) {
        bow_word[j] = e.first;
        bow_value[j] = e.second;
        ++j;
    }
    *bow_n = j;
    j = 0;
    int c = 0;
    for (auto& e : fv) {
        fv_node[j] = e.first;
        for (unsigned i : e.second) fv_idx[c++] = i;
        fv_off[++j] = c;
    }
    *fv_n = j;
    return 0;
}
