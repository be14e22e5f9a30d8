// ORACLE -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the rules).
//
// The sparse solver g2o's LinearSolverEigen hands the reduced pose system to
// (Thirdparty/g2o/g2o/solvers/linear_solver_eigen.h:58-121, chosen by
// src/Optimizer.cc:1341-1343, _blockOrdering = false), restated from Eigen 3.3
// (absent here; not vendored by the reference -- the version ORB-SLAM2-era
// builds link, 3.2 and 3.3 agree on every path below for the matrices g2o
// builds, whose diagonal is always structurally present):
//   fillSparseMatrix   the upper triangle of every Hschur block as triplets ->
//                      column-major CCS, rows sorted, explicit zeros kept;
//   analyzePattern     SimplicialCholeskyBase::ordering: AMDOrdering on the
//                      full symmetric pattern (a + a^T, diagonal kept) =
//                      internal::minimum_degree_ordering (Eigen's port of
//                      CSparse cs_amd: dense rows absorbed into element n,
//                      approximate external degrees, aggressive absorption,
//                      hash-bucket supervariables, postordered assembly tree),
//                      then ap = a.selfadjointView<Upper>().twistedBy(P)
//                      (permute_symm_to_symm: ap's column entries in the order
//                      of the source traversal, NOT sorted), then
//                      analyzePattern_preordered (elimination tree, column
//                      counts);
//   factorize          the same permutation of the values, then
//                      factorize_preordered<DoLDLT>: the up-looking LDL^T of
//                      Tim Davis' LDL -- row k's pattern from elimination-tree
//                      walks in ap's entry order (a topological order),
//                      y[Li] -= Lx * y_i, l_ki = y_i / D_i, d -= l_ki * y_i;
//                      failure on an exact zero pivot;
//   solve              x = P b; L x = x (column-oriented forward substitution,
//                      rows ascending, columns with x_i == 0 skipped);
//                      x = D^-1 x as (1 / d_i) * x_i (asDiagonal().inverse());
//                      L^T x = x (row-oriented backward substitution, rows
//                      ascending); x = P^-1 x.
// Parity unpinned: Eigen is not in this image; checked by
// tests/test_oracle_lba.py (permutations, forced orderings, residuals).
#pragma once
#include <algorithm>
#include <cmath>
#include <vector>

// ORACLE_NS: the namespace of the g2o / Eigen restatement -- "oracle", or "oracle_fma" when the Makefile compiles
// pose_oracle.cpp / lba_oracle.cpp a second time with GCC's FP contraction (the FMA diagnostic mode)
#ifndef ORACLE_NS
#define ORACLE_NS oracle
#endif

namespace ORACLE_NS {
namespace eigen_sparse {

inline int amd_flip(int i) { return -i - 2; }

inline int amd_wclear(int mark, int lemax, int* w, int n) {
    if (mark < 2 || (mark + lemax < 0)) {
        for (int k = 0; k < n; k++)
            if (w[k] != 0) w[k] = 1;
        mark = 2;
    }
    return mark;
}

// depth-first search and postorder of a tree rooted at node j
inline int amd_tdfs(int j, int k, int* head, const int* next, int* post, int* stack) {
    int top = 0;
    stack[0] = j;
    while (top >= 0) {
        const int p = stack[top];
        const int i = head[p];
        if (i == -1) {
            top--;
            post[k++] = p;
        } else {
            head[p] = next[i];
            stack[++top] = i;
        }
    }
    return k;
}

// Eigen::internal::minimum_degree_ordering.  Cp / Ci: the full symmetric pattern (diagonal included, rows of
// every column sorted), consumed.  perm[k] = the node eliminated k-th (Eigen's "inverse permutation" m_Pinv).
inline void minimum_degree_ordering(int n, std::vector<int> Cp, std::vector<int> Ci, std::vector<int>& perm) {
    int d, dk, dext, lemax = 0, e, elenk, eln, i, j, k, k1, k2, k3, jlast, ln, dense, nzmax, mindeg = 0, nvi, nvj,
                     nvk, mark, wnvi, ok, nel = 0, p, p1, p2, p3, p4, pj, pk, pk1, pk2, pn, q, t, h;
    dense = std::max(16, (int)(10 * std::sqrt((double)n)));
    dense = std::min(n - 2, dense);
    int cnz = Cp[n];
    perm.assign(n + 1, 0);
    t = cnz + cnz / 5 + 2 * n;
    Ci.resize(t);
    std::vector<int> W(8 * (n + 1));
    int* len = &W[0];
    int* nv = &W[n + 1];
    int* next = &W[2 * (n + 1)];
    int* head = &W[3 * (n + 1)];
    int* elen = &W[4 * (n + 1)];
    int* degree = &W[5 * (n + 1)];
    int* w = &W[6 * (n + 1)];
    int* hhead = &W[7 * (n + 1)];
    int* last = perm.data();
    for (k = 0; k < n; k++) len[k] = Cp[k + 1] - Cp[k];
    len[n] = 0;
    nzmax = t;
    for (i = 0; i <= n; i++) {
        head[i] = -1;
        last[i] = -1;
        next[i] = -1;
        hhead[i] = -1;
        nv[i] = 1;
        w[i] = 1;
        elen[i] = 0;
        degree[i] = len[i];
    }
    mark = amd_wclear(0, 0, w, n);
    // degree lists
    for (i = 0; i < n; i++) {
        bool has_diag = false;
        for (p = Cp[i]; p < Cp[i + 1]; ++p)
            if (Ci[p] == i) {
                has_diag = true;
                break;
            }
        d = degree[i];
        if (d == 1 && has_diag) {  // empty node
            elen[i] = -2;
            nel++;
            Cp[i] = -1;
            w[i] = 0;
        } else if (d > dense || !has_diag) {  // dense: absorbed into element n
            nv[i] = 0;
            elen[i] = -1;
            nel++;
            Cp[i] = amd_flip(n);
            nv[n]++;
        } else {
            if (head[d] != -1) last[head[d]] = i;
            next[i] = head[d];
            head[d] = i;
        }
    }
    elen[n] = -2;
    Cp[n] = -1;
    w[n] = 0;
    while (nel < n) {
        // node of minimum approximate degree
        for (k = -1; mindeg < n && (k = head[mindeg]) == -1; mindeg++) {
        }
        if (next[k] != -1) last[next[k]] = -1;
        head[mindeg] = next[k];
        elenk = elen[k];
        nvk = nv[k];
        nel += nvk;
        // garbage collection
        if (elenk > 0 && cnz + mindeg >= nzmax) {
            for (j = 0; j < n; j++) {
                if ((p = Cp[j]) >= 0) {
                    Cp[j] = Ci[p];
                    Ci[p] = amd_flip(j);
                }
            }
            for (q = 0, p = 0; p < cnz;) {
                if ((j = amd_flip(Ci[p++])) >= 0) {
                    Ci[q] = Cp[j];
                    Cp[j] = q++;
                    for (k3 = 0; k3 < len[j] - 1; k3++) Ci[q++] = Ci[p++];
                }
            }
            cnz = q;
        }
        // new element
        dk = 0;
        nv[k] = -nvk;
        p = Cp[k];
        pk1 = (elenk == 0) ? p : cnz;
        pk2 = pk1;
        for (k1 = 1; k1 <= elenk + 1; k1++) {
            if (k1 > elenk) {
                e = k;
                pj = p;
                ln = len[k] - elenk;
            } else {
                e = Ci[p++];
                pj = Cp[e];
                ln = len[e];
            }
            for (k2 = 1; k2 <= ln; k2++) {
                i = Ci[pj++];
                if ((nvi = nv[i]) <= 0) continue;
                dk += nvi;
                nv[i] = -nvi;
                Ci[pk2++] = i;
                if (next[i] != -1) last[next[i]] = last[i];
                if (last[i] != -1)
                    next[last[i]] = next[i];
                else
                    head[degree[i]] = next[i];
            }
            if (e != k) {
                Cp[e] = amd_flip(k);
                w[e] = 0;
            }
        }
        if (elenk != 0) cnz = pk2;
        degree[k] = dk;
        Cp[k] = pk1;
        len[k] = pk2 - pk1;
        elen[k] = -2;
        // set differences
        mark = amd_wclear(mark, lemax, w, n);
        for (pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            if ((eln = elen[i]) <= 0) continue;
            nvi = -nv[i];
            wnvi = mark - nvi;
            for (p = Cp[i]; p <= Cp[i] + eln - 1; p++) {
                e = Ci[p];
                if (w[e] >= mark)
                    w[e] -= nvi;
                else if (w[e] != 0)
                    w[e] = degree[e] + wnvi;
            }
        }
        // degree update
        for (pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            p1 = Cp[i];
            p2 = p1 + elen[i] - 1;
            pn = p1;
            for (h = 0, d = 0, p = p1; p <= p2; p++) {
                e = Ci[p];
                if (w[e] != 0) {
                    dext = w[e] - mark;
                    if (dext > 0) {
                        d += dext;
                        Ci[pn++] = e;
                        h += e;
                    } else {
                        Cp[e] = amd_flip(k);  // aggressive absorption
                        w[e] = 0;
                    }
                }
            }
            elen[i] = pn - p1 + 1;
            p3 = pn;
            p4 = p1 + len[i];
            for (p = p2 + 1; p < p4; p++) {
                j = Ci[p];
                if ((nvj = nv[j]) <= 0) continue;
                d += nvj;
                Ci[pn++] = j;
                h += j;
            }
            if (d == 0) {  // mass elimination
                Cp[i] = amd_flip(k);
                nvi = -nv[i];
                dk -= nvi;
                nvk += nvi;
                nel += nvi;
                nv[i] = 0;
                elen[i] = -1;
            } else {
                degree[i] = std::min(degree[i], d);
                Ci[pn] = Ci[p3];
                Ci[p3] = Ci[p1];
                Ci[p1] = k;
                len[i] = pn - p1 + 1;
                h %= n;
                next[i] = hhead[h];
                hhead[h] = i;
                last[i] = h;
            }
        }
        degree[k] = dk;
        lemax = std::max(lemax, dk);
        mark = amd_wclear(mark + lemax, lemax, w, n);
        // supernode detection
        for (pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            if (nv[i] >= 0) continue;
            h = last[i];
            i = hhead[h];
            hhead[h] = -1;
            for (; i != -1 && next[i] != -1; i = next[i], mark++) {
                ln = len[i];
                eln = elen[i];
                for (p = Cp[i] + 1; p <= Cp[i] + ln - 1; p++) w[Ci[p]] = mark;
                jlast = i;
                for (j = next[i]; j != -1;) {
                    ok = (len[j] == ln) && (elen[j] == eln);
                    for (p = Cp[j] + 1; ok && p <= Cp[j] + ln - 1; p++)
                        if (w[Ci[p]] != mark) ok = 0;
                    if (ok) {
                        Cp[j] = amd_flip(i);
                        nv[i] += nv[j];
                        nv[j] = 0;
                        elen[j] = -1;
                        j = next[j];
                        next[jlast] = j;
                    } else {
                        jlast = j;
                        j = next[j];
                    }
                }
            }
        }
        // finalize the new element
        for (p = pk1, pk = pk1; pk < pk2; pk++) {
            i = Ci[pk];
            if ((nvi = -nv[i]) <= 0) continue;
            nv[i] = nvi;
            d = degree[i] + dk - nvi;
            d = std::min(d, n - nel - nvi);
            if (head[d] != -1) last[head[d]] = i;
            next[i] = head[d];
            last[i] = -1;
            head[d] = i;
            mindeg = std::min(mindeg, d);
            degree[i] = d;
            Ci[p++] = i;
        }
        nv[k] = nvk;
        if ((len[k] = p - pk1) == 0) {
            Cp[k] = -1;
            w[k] = 0;
        }
        if (elenk != 0) cnz = p;
    }
    // postorder the assembly tree
    for (i = 0; i < n; i++) Cp[i] = amd_flip(Cp[i]);
    for (j = 0; j <= n; j++) head[j] = -1;
    for (j = n; j >= 0; j--) {
        if (nv[j] > 0) continue;
        next[j] = head[Cp[j]];
        head[Cp[j]] = j;
    }
    for (e = n; e >= 0; e--) {
        if (nv[e] <= 0) continue;
        if (Cp[e] != -1) {
            next[e] = head[Cp[e]];
            head[Cp[e]] = e;
        }
    }
    for (k = 0, i = 0; i <= n; i++)
        if (Cp[i] == -1) k = amd_tdfs(i, k, head, next, perm.data(), w);
    perm.resize(n);
}

// SimplicialLDLT<SparseMatrix<double>, Upper> over a fixed upper pattern (a: column-major CCS, rows of each
// column sorted, every entry with row <= column).
struct SimplicialLDLT {
    int n = 0;
    std::vector<int> Pinv, P;   // Pinv[k] = old index of new k (AMD); P[old] = new
    std::vector<int> apP, apI;  // ap = P a P^T (upper): column c's rows in permute_symm_to_symm order
    std::vector<int> apSrc;     // per ap entry: the index of its value in a's CCS value array
    std::vector<int> parent, nzc, Lp;
    std::vector<int> Li;
    std::vector<double> Lx, D;

    void analyze(int n_, const std::vector<int>& Ap, const std::vector<int>& Ai) {
        n = n_;
        // full symmetric pattern C = a + a^T (sorted columns: permute_symm_to_fullsymm, then A^T + A)
        std::vector<std::vector<int>> cols(n);
        for (int j = 0; j < n; j++)
            for (int p = Ap[j]; p < Ap[j + 1]; p++) {
                const int i = Ai[p];
                cols[j].push_back(i);
                if (i != j) cols[i].push_back(j);
            }
        std::vector<int> Cp(n + 1, 0), Ci;
        for (int j = 0; j < n; j++) {
            std::sort(cols[j].begin(), cols[j].end());
            cols[j].erase(std::unique(cols[j].begin(), cols[j].end()), cols[j].end());
            Cp[j + 1] = Cp[j] + (int)cols[j].size();
            Ci.insert(Ci.end(), cols[j].begin(), cols[j].end());
        }
        minimum_degree_ordering(n, Cp, Ci, Pinv);
        P.assign(n, 0);
        for (int k = 0; k < n; k++) P[Pinv[k]] = k;
        // permute_symm_to_symm<Upper, Upper>: count per destination column, then append in source order
        std::vector<int> count(n, 0);
        for (int j = 0; j < n; j++)
            for (int p = Ap[j]; p < Ap[j + 1]; p++) count[std::max(P[Ai[p]], P[j])]++;
        apP.assign(n + 1, 0);
        for (int j = 0; j < n; j++) apP[j + 1] = apP[j] + count[j];
        apI.assign(apP[n], 0);
        apSrc.assign(apP[n], 0);
        for (int j = 0; j < n; j++) count[j] = apP[j];
        for (int j = 0; j < n; j++)
            for (int p = Ap[j]; p < Ap[j + 1]; p++) {
                const int ip = P[Ai[p]], jp = P[j];
                const int k = count[std::max(ip, jp)]++;
                apI[k] = std::min(ip, jp);
                apSrc[k] = p;
            }
        // analyzePattern_preordered: elimination tree and column counts
        parent.assign(n, -1);
        nzc.assign(n, 0);
        std::vector<int> tags(n, 0);
        for (int k = 0; k < n; k++) {
            parent[k] = -1;
            tags[k] = k;
            nzc[k] = 0;
            for (int p = apP[k]; p < apP[k + 1]; p++) {
                int i = apI[p];
                if (i < k)
                    for (; tags[i] != k; i = parent[i]) {
                        if (parent[i] == -1) parent[i] = k;
                        nzc[i]++;
                        tags[i] = k;
                    }
            }
        }
        Lp.assign(n + 1, 0);
        for (int k = 0; k < n; k++) Lp[k + 1] = Lp[k] + nzc[k];
        Li.assign(Lp[n], 0);
        Lx.assign(Lp[n], 0.0);
        D.assign(n, 0.0);
    }

    // Ax: a's values in its CCS order.  false on a zero pivot (Eigen's NumericalIssue).
    bool factorize(const std::vector<double>& Ax) {
        std::vector<double> y(n, 0.0);
        std::vector<int> pattern(n, 0), tags(n, 0), cnt(n, 0);
        for (int k = 0; k < n; k++) {
            y[k] = 0.0;
            int top = n;
            tags[k] = k;
            cnt[k] = 0;
            for (int p = apP[k]; p < apP[k + 1]; p++) {
                int i = apI[p];
                if (i <= k) {
                    y[i] += Ax[apSrc[p]];
                    int len;
                    for (len = 0; tags[i] != k; i = parent[i]) {
                        pattern[len++] = i;
                        tags[i] = k;
                    }
                    while (len > 0) pattern[--top] = pattern[--len];
                }
            }
            double d = y[k] * 1.0 + 0.0;  // m_shiftScale, m_shiftOffset
            y[k] = 0.0;
            for (; top < n; ++top) {
                const int i = pattern[top];
                const double yi = y[i];
                y[i] = 0.0;
                const double l_ki = yi / D[i];
                const int p2 = Lp[i] + cnt[i];
                int p;
                for (p = Lp[i]; p < p2; ++p) y[Li[p]] -= Lx[p] * yi;
                d -= l_ki * yi;
                Li[p] = k;
                Lx[p] = l_ki;
                ++cnt[i];
            }
            D[k] = d;
            if (d == 0.0) return false;
        }
        return true;
    }

    void solve(const double* b, double* x) const {
        std::vector<double> t(n);
        for (int i = 0; i < n; i++) t[P[i]] = b[i];
        if (Lp[n] > 0)
            for (int i = 0; i < n; i++) {
                const double tmp = t[i];
                if (tmp != 0.0)
                    for (int p = Lp[i]; p < Lp[i + 1]; p++) t[Li[p]] -= tmp * Lx[p];
            }
        for (int i = 0; i < n; i++) t[i] = (1.0 / D[i]) * t[i];
        if (Lp[n] > 0)
            for (int i = n - 1; i >= 0; i--) {
                double tmp = t[i];
                for (int p = Lp[i]; p < Lp[i + 1]; p++) tmp -= Lx[p] * t[Li[p]];
                t[i] = tmp;
            }
        for (int k = 0; k < n; k++) x[Pinv[k]] = t[k];
    }
};

}  // namespace eigen_sparse
}  // namespace oracle
