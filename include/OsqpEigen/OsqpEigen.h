/*
 * include/OsqpEigen/OsqpEigen.h — the osqp-eigen call surface, Eigen-typed, over the MI355X C ABI.
 *
 * LukeSchmitt96/solveMPC includes "OsqpEigen/OsqpEigen.h" (include/ModelPredictiveControlAPI.h:11) and
 * owns one `OsqpEigen::Solver solver` (:144).  With this directory on the include path ahead of the
 * real osqp-eigen, that member runs its QP on a gfx950 device through include/mpcq.h, and the
 * reference's call shapes below compile against it (shown by tests/cpp/reference_caller.cpp; the
 * reference file itself also needs Eigen's unsupported MatrixFunctions, absent here: DESIGN.md section 7):
 *
 *   solver.settings()->setVerbosity(verbose); solver.settings()->setWarmStart(true);   (cpp:51-52)
 *   solver.data()->setNumberOfVariables(n); ...->setNumberOfConstraints(m);           (cpp:54-55)
 *   solver.data()->setHessianMatrix(H)             H: Eigen::SparseMatrix<double>     (cpp:57)
 *   solver.data()->setGradient(f)                  f: Eigen::Matrix<double, N, 1>     (cpp:58)
 *   solver.data()->setLinearConstraintsMatrix(Gbar) Gbar: Eigen::SparseMatrix<double> (cpp:59)
 *   solver.data()->setLowerBound(lb) / setUpperBound(ub)                              (cpp:60-61)
 *   solver.initSolver()                                                                (cpp:64)
 *   solver.updateGradient(f); solver.updateUpperBound(W0 + Sbar*X + Ku*U)  (expressions) (cpp:96,99)
 *   solver.solve()                                 -> bool, true only for OSQP_SOLVED  (cpp:102)
 *   U += solver.getSolution().block<N_C, 1>(0, 0)  getSolution(): const Eigen::VectorXd& (cpp:105)
 *
 * Header-only and templated on the caller's Eigen: the library itself (libmpcq.so) has no Eigen in
 * its interface.  Every bool-returning call is false on any error, as osqp-eigen's are; the reason
 * is in lastError() (mpcq_last_error()).  Sparse matrices are densified (the reference stores its
 * H and Gbar with every entry, explicit zeros included: ModelPredictiveControlAPI.cpp:254-263,
 * 339-347); the Hessian's upper triangle is read, as osqp-eigen passes triangularView<Upper>.
 * One QP per Solver (the reference's shape); the batched form is the C ABI itself.
 */
#ifndef SOLVEMPC_AMD_OSQPEIGEN_H
#define SOLVEMPC_AMD_OSQPEIGEN_H

#include <Eigen/Dense>
#include <Eigen/Sparse>

#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "../mpcq.h"

namespace OsqpEigen {

/* osqp-eigen Settings (OSQP v0.6 defaults via mpcq_default_settings).  Method names keep
 * osqp-eigen's spelling, typos included (setPrimalInfeasibilityTollerance, setScaledTerimination). */
class Settings {
public:
    Settings() { mpcq_default_settings(&s_); }
    void resetDefaultSettings() { mpcq_default_settings(&s_); polish_ = false; }
    void setRho(double v) { s_.rho = v; }
    void setSigma(double v) { s_.sigma = v; }
    void setScaling(int v) { s_.scaling = v; }
    void setAdaptiveRho(bool v) { s_.adaptive_rho = v; }
    void setAdaptiveRhoInterval(int v) { s_.adaptive_rho_interval = v; }
    void setAdaptiveRhoTolerance(double v) { s_.adaptive_rho_tolerance = v; }
    void setAdaptiveRhoFraction(double v) { s_.adaptive_rho_fraction = v; }
    void setMaxIteration(int v) { s_.max_iter = v; }
    void setAbsoluteTolerance(double v) { s_.eps_abs = v; }
    void setRelativeTolerance(double v) { s_.eps_rel = v; }
    void setPrimalInfeasibilityTollerance(double v) { s_.eps_prim_inf = v; }
    void setDualInfeasibilityTollerance(double v) { s_.eps_dual_inf = v; }
    void setAlpha(double v) { s_.alpha = v; }
    void setLinearSystemSolver(int) {}  // the device factorisation replaces QDLDL / MKL Pardiso
    void setDelta(double) {}            // polishing only
    void setPolish(bool v) { polish_ = v; }  // not implemented: initSolver() fails when set
    void setPolishRefineIter(int) {}
    void setVerbosity(bool v) { s_.verbose = v; }
    void setScaledTerimination(bool v) { s_.scaled_termination = v; }
    void setCheckTermination(int v) { s_.check_termination = v; }
    void setWarmStart(bool v) { s_.warm_start = v; }
    void setTimeLimit(double) {}  // OSQP's time limit is a PROFILING feature; unsupported, ignored
    const mpcq_settings &getSettings() const { return s_; }
    bool polish() const { return polish_; }

private:
    mpcq_settings s_;
    bool polish_ = false;
};

/* osqp-eigen Data: sizes first, then the problem arrays (copied at set time). */
class Data {
public:
    void setNumberOfVariables(int n) { n_ = n; }
    void setNumberOfConstraints(int m) { m_ = m; }
    int getNumberOfVariables() const { return n_; }
    int getNumberOfConstraints() const { return m_; }

    template <typename Derived>
    bool setHessianMatrix(const Eigen::SparseCompressedBase<Derived> &H)
    {
        if (n_ < 0 || H.rows() != n_ || H.cols() != n_) return false;
        P_ = Eigen::MatrixXd(H.derived()).template triangularView<Eigen::Upper>();
        has_ |= kP;
        return true;
    }
    template <typename Derived>
    bool setLinearConstraintsMatrix(const Eigen::SparseCompressedBase<Derived> &A)
    {
        if (n_ < 0 || m_ < 0 || A.rows() != m_ || A.cols() != n_) return false;
        A_ = Eigen::MatrixXd(A.derived());
        has_ |= kA;
        return true;
    }
    template <typename Derived>
    bool setGradient(const Eigen::MatrixBase<Derived> &q)
    {
        if (n_ < 0 || q.size() != n_) return false;
        q_ = q;
        has_ |= kQ;
        return true;
    }
    template <typename Derived>
    bool setLowerBound(const Eigen::MatrixBase<Derived> &l)
    {
        if (m_ < 0 || l.size() != m_) return false;
        l_ = l;
        has_ |= kL;
        return true;
    }
    template <typename Derived>
    bool setUpperBound(const Eigen::MatrixBase<Derived> &u)
    {
        if (m_ < 0 || u.size() != m_) return false;
        u_ = u;
        has_ |= kU;
        return true;
    }
    bool isSet() const { return has_ == (kP | kQ | kA | kL | kU) || (m_ == 0 && (has_ & (kP | kQ)) == (kP | kQ)); }
    void clearHessianMatrix() { has_ &= ~kP; }
    void clearLinearConstraintsMatrix() { has_ &= ~kA; }

private:
    friend class Solver;
    enum { kP = 1, kQ = 2, kA = 4, kL = 8, kU = 16 };
    int n_ = -1, m_ = -1, has_ = 0;
    Eigen::MatrixXd P_, A_;  // column-major (Eigen default); the C ABI reads row-major
    Eigen::VectorXd q_, l_, u_;
};

class Solver {
public:
    explicit Solver(int device = 0) : settings_(new Settings()), data_(new Data()), device_(device) {}
    ~Solver() { clearSolver(); }
    Solver(const Solver &) = delete;
    Solver &operator=(const Solver &) = delete;

    const std::unique_ptr<Settings> &settings() const { return settings_; }
    const std::unique_ptr<Data> &data() const { return data_; }

    /* osqp_setup on the device (mpcq_create + mpcq_setup: Ruiz scaling, KKT basis) */
    bool initSolver()
    {
        if (ctx_) return fail("initSolver: the solver is already initialised");
        if (settings_->polish()) return fail("initSolver: solution polishing is not supported");
        const Data &d = *data_;
        if (!d.isSet()) return fail("initSolver: the problem data are not set");
        mpcq_dims dims{d.n_, d.m_, 1, 1, MPCQ_F64, device_};
        if (mpcq_create(&dims, &settings_->getSettings(), &ctx_) != MPCQ_OK) {
            ctx_ = nullptr;
            return fail("initSolver");
        }
        const RowMajor P = d.P_, A = d.m_ ? RowMajor(d.A_) : RowMajor(1, d.n_);
        const Eigen::VectorXd l = d.m_ ? d.l_ : Eigen::VectorXd(1), u = d.m_ ? d.u_ : Eigen::VectorXd(1);
        if (mpcq_setup(ctx_, P.data(), d.q_.data(), A.data(), l.data(), u.data()) != MPCQ_OK) {
            fail("initSolver");
            clearSolver();
            return false;
        }
        x_ = Eigen::VectorXd::Zero(d.n_);
        y_ = Eigen::VectorXd::Zero(d.m_);
        l_ = d.l_;
        u_ = d.u_;
        return true;
    }
    bool isInitialized() const { return ctx_ != nullptr; }
    void clearSolver()
    {
        if (ctx_) mpcq_destroy(ctx_);
        ctx_ = nullptr;
    }

    /* osqp_update_lin_cost / osqp_update_{upper,lower}_bound / osqp_update_bounds.  Eigen::Ref
     * evaluates expressions such as W0 + Sbar*X + Ku*U (ModelPredictiveControlAPI.cpp:99). */
    bool updateGradient(const Eigen::Ref<const Eigen::VectorXd> &q)
    {
        if (!ctx_ || q.size() != data_->n_) return fail("updateGradient: not initialised or wrong size");
        const Eigen::VectorXd v = q;
        return mpcq_update_lin_cost(ctx_, v.data()) == MPCQ_OK || fail("updateGradient");
    }
    bool updateUpperBound(const Eigen::Ref<const Eigen::VectorXd> &u)
    {
        if (!ctx_ || u.size() != data_->m_) return fail("updateUpperBound: not initialised or wrong size");
        const Eigen::VectorXd v = u;  // (osqp_update_upper_bound rejects u < l)
        if ((v.array() < l_.array()).any()) return fail("updateUpperBound: upper bound below the lower bound");
        if (mpcq_update_upper_bound(ctx_, v.data()) != MPCQ_OK) return fail("updateUpperBound");
        u_ = v;
        return true;
    }
    bool updateLowerBound(const Eigen::Ref<const Eigen::VectorXd> &l)
    {
        if (!ctx_ || l.size() != data_->m_) return fail("updateLowerBound: not initialised or wrong size");
        const Eigen::VectorXd v = l;
        if ((v.array() > u_.array()).any()) return fail("updateLowerBound: lower bound above the upper bound");
        if (mpcq_update_lower_bound(ctx_, v.data()) != MPCQ_OK) return fail("updateLowerBound");
        l_ = v;
        return true;
    }
    bool updateBounds(const Eigen::Ref<const Eigen::VectorXd> &l, const Eigen::Ref<const Eigen::VectorXd> &u)
    {
        if (!ctx_ || l.size() != data_->m_ || u.size() != data_->m_) return fail("updateBounds: wrong size");
        const Eigen::VectorXd lv = l, uv = u;
        if ((lv.array() > uv.array()).any()) return fail("updateBounds: lower bound above the upper bound");
        if (mpcq_update_bounds(ctx_, lv.data(), uv.data()) != MPCQ_OK) return fail("updateBounds");
        l_ = lv;
        u_ = uv;
        return true;
    }
    /* osqp_warm_start(x, y) */
    bool setWarmStart(const Eigen::Ref<const Eigen::VectorXd> &x, const Eigen::Ref<const Eigen::VectorXd> &y)
    {
        if (!ctx_ || x.size() != data_->n_ || y.size() != data_->m_) return fail("setWarmStart: wrong size");
        const Eigen::VectorXd xv = x, yv = y;
        return mpcq_warm_start(ctx_, xv.data(), yv.data()) == MPCQ_OK || fail("setWarmStart");
    }

    /* osqp_solve; osqp-eigen v0.6 returns false on an error or any status but OSQP_SOLVED.  A
     * u < l from the last bound update surfaces here as MPCQ_INVALID_BOUNDS (false). */
    bool solve()
    {
        if (!ctx_) return fail("solve: the solver is not initialised");
        if (mpcq_solve(ctx_, nullptr) != MPCQ_OK) return fail("solve");
        double rho = 0.0;
        if (mpcq_get_info(ctx_, &status_, &iter_, &rho) != MPCQ_OK) return fail("solve");
        if (mpcq_get_solution(ctx_, x_.data()) != MPCQ_OK) return fail("solve");
        if (data_->m_ && mpcq_get_dual(ctx_, y_.data()) != MPCQ_OK) return fail("solve");
        return status_ == MPCQ_SOLVED;
    }
    const Eigen::VectorXd &getSolution() const { return x_; }
    const Eigen::VectorXd &getDualSolution() const { return y_; }
    int getStatus() const { return status_; }
    int getIterations() const { return iter_; }
    const std::string &lastError() const { return err_; }

private:
    typedef Eigen::Matrix<double, Eigen::Dynamic, Eigen::Dynamic, Eigen::RowMajor> RowMajor;
    bool fail(const char *where)
    {
        err_ = std::string(where) + ": " + mpcq_last_error();
        if (settings_->getSettings().verbose) std::fprintf(stderr, "[OsqpEigen] %s\n", err_.c_str());
        return false;
    }
    std::unique_ptr<Settings> settings_;
    std::unique_ptr<Data> data_;
    int device_;
    mpcq_ctx *ctx_ = nullptr;
    Eigen::VectorXd x_, y_, l_, u_;  // solution; current bounds (the update calls' u >= l check)
    int status_ = MPCQ_UNSOLVED, iter_ = 0;
    std::string err_;
};

}  // namespace OsqpEigen

#endif  // SOLVEMPC_AMD_OSQPEIGEN_H
