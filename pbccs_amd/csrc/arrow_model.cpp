// pbccs_amd/csrc/arrow_model.cpp -- see arrow_model.hpp.
#include "arrow_model.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <stdexcept>

namespace pbccs {

namespace {

// SNR polynomial fits per context (ContextParameterProvider.cpp:20-61): for each context the
// log-odds of {dark (deletion), match, stick} against branch, as a cubic in the channel SNR.
const char kContextChannel[8] = {'A', 'C', 'G', 'T', 'A', 'C', 'G', 'T'};
const double kPoly[8][3][4] = {
    // AA
    {{3.76122480667588, -0.536010820176981, 0.0275375059387171, -0.000470200724345621},
     {3.57517725358548, -0.0257545295375707, -0.000163673803286944, 5.3256984681724e-06},
     {0.858421613302247, -0.0276654216841666, -8.85549766507732e-05, -4.85355908595337e-05}},
    // CC
    {{5.66725538674764, -1.10462196933913, 0.0879811093908922, -0.00259393800835979},
     {4.11682756767018, -0.124758322644639, 0.00659795177909886, -0.000361914629195461},
     {3.17103818507405, -0.729020290806687, 0.0749784690396837, -0.00262779517495421}},
    // GG
    {{3.81920778703052, -0.540309003502589, 0.0389569264893982, -0.000901245733796236},
     {3.31322216145728, 0.123514009118836, -0.00807401406655071, 0.000230843924466035},
     {2.06006877520527, -0.451486652688621, 0.0375212898173045, -0.000937676250926241}},
    // TT
    {{5.39308368236762, -1.32931568057267, 0.107844580241936, -0.00316462903462847},
     {4.21031404956015, -0.347546363361823, 0.0293839179303896, -0.000893802212450644},
     {2.33143889851302, -0.586068444099136, 0.040044954697795, -0.000957298861394191}},
    // NA
    {{2.35936060895653, -0.463630601682986, 0.0179206897766131, -0.000230839937063052},
     {3.22847830625841, -0.0886820214931539, 0.00555981712798726, -0.000137686231186054},
     {-0.101031042923432, -0.0138783767832632, -0.00153408019582419, 7.66780338484727e-06}},
    // NC
    {{5.956054206161, -1.71886470811695, 0.153315470604752, -0.00474488595513198},
     {3.89418464416296, -0.174182841558867, 0.0171719290275442, -0.000653629721359769},
     {2.40532887070852, -0.652606650098156, 0.0688783864119339, -0.00246479494650594}},
    // NG
    {{3.53508304630569, -0.788027301381263, 0.0469367803413207, -0.00106221924705805},
     {2.85440184222226, 0.166346531056167, -0.0166161828155307, 0.000439492705370092},
     {0.238188180807376, 0.0589443522886522, -0.0123401045958974, 0.000336854126836293}},
    // NT
    {{5.36199280681367, -1.46099908985536, 0.126755291030074, -0.0039102734460725},
     {3.41597143103046, -0.066984162951578, 0.0138944877787003, -0.000558939998921912},
     {1.37371376794871, -0.246963827944892, 0.0209674231346363, -0.000684856715039738}},
};

int channel(char c) { return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3; }

}  // namespace

void transition_table(const double snr[4], TransParams out[8])
{
    for (int k = 0; k < 8; ++k) {
        const double x = snr[channel(kContextChannel[k])];
        const double x2 = x * x;
        const double x3 = x2 * x;
        double odds[3];
        double denom = 1.0;
        for (int row = 0; row < 3; ++row) {
            const double* c = kPoly[k][row];
            const double eta = c[0] + x * c[1] + x2 * c[2] + x3 * c[3];
            odds[row] = std::exp(eta);
            denom += odds[row];
        }
        TransParams p;
        p.branch = 1.0 / denom;
        p.deletion = odds[0] / denom;
        p.match = odds[1] / denom;
        p.stick = odds[2] / denom;
        out[k] = p;
    }
}

void device_context_table(const TransParams t[8], double out[45])
{
    for (int k = 0; k < 9; ++k) {
        const TransParams p = k < 8 ? t[k] : TransParams();
        out[5 * k + 0] = p.match;
        out[5 * k + 1] = p.stick;
        out[5 * k + 2] = p.branch;
        out[5 * k + 3] = p.deletion;
        out[5 * k + 4] = p.stick / 3.0;   // the recursions' (Stick / 3.0), computed once
    }
}

std::pair<double, double> expected_context_ll(const TransParams& p, double eps)
{
    const double pm = p.match, pd = p.deletion, pb = p.branch, ps = p.stick;
    const double lm = std::log(pm), ld = std::log(pd), lb = std::log(pb), ls = std::log(ps);
    const double third = -std::log(3.0);
    const double eM = (1.0 - eps) * 0.0 + eps * third, e2M = eps * third * third;
    const double eD = 0.0, e2D = eD * eD;
    const double eB = 0.0, e2B = eB * eB;
    const double eS = third, e2S = eS * eS;
    auto moment = [&](double xm, double xd, double xb, double xs, double ym, double yd, double yb, double ys) {
        const double md = (xm + ym) * pm / (pm + pd) + (xd + yd) * pd / (pm + pd);
        const double ins = (xb + yb) * pb / (pb + ps) + (xs + ys) * ps / (pb + ps);
        const double bs = ins * (ps + pb) / (pm + pd);
        return md + bs;
    };
    const double mean = moment(lm, ld, lb, ls, eM, eD, eB, eS);
    const double var = moment(lm * lm, ld * ld, lb * lb, ls * ls, e2M, e2D, e2B, e2S) - mean * mean;
    return {mean, var};
}

int mutation_code(const Mutation& m)
{
    int b = 0;
    if (m.type != 1) b = m.base == 'A' ? 0 : m.base == 'C' ? 1 : m.base == 'G' ? 2 : 3;
    return (m.start << 4) | (m.type << 2) | b;
}

Mutation mutation_from_code(int code)
{
    return Mutation::Make((code >> 2) & 3, code >> 4, "ACGT"[code & 3]);
}

bool is_acgt(const std::string& s)
{
    for (char c : s)
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T') return false;
    return true;
}

std::string reverse_complement(const std::string& s)
{
    std::string r(s.rbegin(), s.rend());
    for (char& c : r) c = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : c;
    return r;
}

long long unique_mutation_count(const std::string& tpl)
{
    if (tpl.empty()) return 0;
    long long n = 8;
    for (size_t p = 1; p < tpl.size(); ++p) n += 6 + (tpl[p] != tpl[p - 1] ? 1 : 0);
    return n;
}

static const char kBases[4] = {'A', 'C', 'G', 'T'};

void unique_mutations(const std::string& tpl, int b, int e, std::vector<int>* codes)
{
    const int L = (int)tpl.size();
    b = std::max(0, std::min(b, L));
    e = std::max(0, std::min(e, L));
    for (int p = b; p < e; ++p) {
        const char prev = p > 0 ? tpl[p - 1] : '-';
        for (int x = 0; x < 4; ++x)
            if (kBases[x] != tpl[p]) codes->push_back((p << 4) | (2 << 2) | x);
        for (int x = 0; x < 4; ++x)
            if (kBases[x] != prev) codes->push_back((p << 4) | (0 << 2) | x);
        if (tpl[p] != prev) codes->push_back((p << 4) | (1 << 2));
    }
}

void nearby_mutations(const std::string& tpl, const std::vector<int>& centerStarts, int nbhd,
                      std::vector<int>* codes)
{
    // The union of Mutations(c - nbhd, c + nbhd) over the centres, in std::set<Mutation> order:
    // by position, then end (insertions end at start), type (DEL < SUB) and base.
    const int L = (int)tpl.size();
    std::vector<char> mark(L + 1, 0);
    for (int c : centerStarts) {
        const int b = std::max(0, std::min(c - nbhd, L));
        const int e = std::max(0, std::min(c + nbhd, L));
        for (int p = b; p < e; ++p) mark[p] = 1;
    }
    for (int p = 0; p < L; ++p) {
        if (!mark[p]) continue;
        const char prev = p > 0 ? tpl[p - 1] : '-';
        for (int x = 0; x < 4; ++x)
            if (kBases[x] != prev) codes->push_back((p << 4) | (0 << 2) | x);
        if (tpl[p] != prev) codes->push_back((p << 4) | (1 << 2));
        for (int x = 0; x < 4; ++x)
            if (kBases[x] != tpl[p]) codes->push_back((p << 4) | (2 << 2) | x);
    }
}

bool apply_mutations(const std::string& tpl, std::vector<Mutation> muts, std::string* out, std::vector<int>* mtp)
{
    std::sort(muts.begin(), muts.end());
    // transcript (MutationsToTranscript, Mutation.cpp:131-170) -> target-to-query map (PairwiseAlignment.cpp:264-297)
    std::string tx;
    int tpos = 0;
    for (const Mutation& m : muts) {
        for (; tpos < m.start; ++tpos) tx.push_back('M');
        if (m.type == 0) tx.push_back('I');
        else if (m.type == 1) { tx.push_back('D'); tpos += 1; }
        else { tx.push_back('R'); tpos += 1; }
    }
    for (; tpos < (int)tpl.size(); ++tpos) tx.push_back('M');
    mtp->clear();
    int q = 0;
    for (char c : tx) {
        if (c == 'M' || c == 'R') { mtp->push_back(q); ++q; }
        else if (c == 'D') mtp->push_back(q);
        else ++q;
    }
    mtp->push_back(q);
    // real edits with a running length offset (ApplyMutations, Mutation.cpp:115-128)
    std::string s(tpl);
    int shift = 0;
    for (const Mutation& m : muts) {
        const int at = m.start + shift;
        if (m.type == 2) {
            if (at < 0 || at >= (int)s.size()) return false;
            s[at] = m.base;
        } else if (m.type == 1) {
            if (at < 0 || at >= (int)s.size()) return false;
            s.erase(at, 1);
        } else {
            // TemplateParameterPair::_ApplyMutationInPlace reads tpl.at(start + 1) after an
            // insertion: inserting at (or past) the end throws in the reference.
            if (at < 0 || at >= (int)s.size()) return false;
            s.insert(s.begin() + at, m.base);
        }
        shift += m.LengthDiff();
    }
    *out = s;
    return true;
}

int probability_to_qv(double p)
{
    if (p < 0.0 || p > 1.0) throw std::invalid_argument("invalid value: probability not in [0,1]");
    if (p == 0.0) p = std::numeric_limits<double>::min();
    return static_cast<int>(std::round(-10.0 * std::log10(p)));
}

}  // namespace pbccs
