// solvempc_amd/cpp/mpcq_solver.hpp — C++ host layer over the C ABI (include/mpcq.h).
//
// Mirrors the osqp-eigen call surface that LukeSchmitt96/solveMPC uses
// (src/ModelPredictiveControlAPI.cpp:51-64 setup, :96-105 per step):
//   solver.settings()->setVerbosity(bool) / setWarmStart(bool)
//   solver.data()->setNumberOfVariables(n) / setNumberOfConstraints(m)
//   solver.data()->setHessianMatrix(H) / setGradient(f) / setLinearConstraintsMatrix(G)
//                 / setLowerBound(l) / setUpperBound(u)                           -> bool
//   solver.initSolver() / updateGradient(f) / updateUpperBound(u) / solve()       -> bool
//   solver.getSolution()                                                          -> const Vector&
// with the same boolean error behaviour (false on any failure; solve() true only for OSQP_SOLVED).
// Eigen is not part of this build: matrices are mpcq::Matrix (column-major, like Eigen's default).
#pragma once

#include <ostream>
#include <string>
#include <vector>

#include "../../include/mpcq.h"

namespace mpcq {

// Dense column-major matrix with the Eigen accessors the reference's code relies on.
class Matrix {
public:
    Matrix() = default;
    Matrix(int rows, int cols, double fill = 0.0) : r_(rows), c_(cols), v_((size_t)rows * cols, fill) {}
    static Matrix Zero(int rows, int cols) { return Matrix(rows, cols); }
    static Matrix Ones(int rows, int cols) { return Matrix(rows, cols, 1.0); }
    int rows() const { return r_; }
    int cols() const { return c_; }
    size_t size() const { return v_.size(); }
    double &operator()(int i, int j) { return v_[(size_t)j * r_ + i]; }
    double operator()(int i, int j) const { return v_[(size_t)j * r_ + i]; }
    double &operator()(int i) { return v_[i]; }
    double operator()(int i) const { return v_[i]; }
    double *data() { return v_.data(); }
    const double *data() const { return v_.data(); }
    void resize(int rows, int cols) { r_ = rows; c_ = cols; v_.assign((size_t)rows * cols, 0.0); }
    // row-major copy (the C ABI's layout)
    std::vector<double> row_major() const;
    static Matrix from_row_major(int rows, int cols, const double *p);
    Matrix transpose() const;
    Matrix operator*(const Matrix &b) const;

private:
    int r_ = 0, c_ = 0;
    std::vector<double> v_;
};

// Printed as Eigen's default IOFormat prints a matrix (the reference's -v dumps,
// ModelPredictiveControlAPI.cpp:118-176,210-243,265-321): every coefficient right-aligned to the
// widest one at the stream's precision, columns separated by one space, rows by newlines.
std::ostream &operator<<(std::ostream &os, const Matrix &m);

using Vector = std::vector<double>;

// osqp-eigen-shaped solver for ONE QP, running on the gfx950 device through the C ABI.
class Solver {
public:
    class Settings {
    public:
        void setVerbosity(bool v) { s_.verbose = v; }
        void setWarmStart(bool w) { s_.warm_start = w; }
        void setRho(double r) { s_.rho = r; }
        void setSigma(double s) { s_.sigma = s; }
        void setAlpha(double a) { s_.alpha = a; }
        void setMaxIteration(int i) { s_.max_iter = i; }
        void setAbsoluteTolerance(double e) { s_.eps_abs = e; }
        void setRelativeTolerance(double e) { s_.eps_rel = e; }
        void setPrimalInfeasibilityTollerance(double e) { s_.eps_prim_inf = e; }
        void setDualInfeasibilityTollerance(double e) { s_.eps_dual_inf = e; }
        void setScaling(int s) { s_.scaling = s; }
        void setAdaptiveRho(bool a) { s_.adaptive_rho = a; }
        void setAdaptiveRhoInterval(int i) { s_.adaptive_rho_interval = i; }
        void setAdaptiveRhoTolerance(double t) { s_.adaptive_rho_tolerance = t; }
        void setCheckTermination(int c) { s_.check_termination = c; }
        void setScaledTerimination(bool s) { s_.scaled_termination = s; }
        const mpcq_settings &raw() const { return s_; }
        Settings() { mpcq_default_settings(&s_); }

    private:
        mpcq_settings s_;
    };

    class Data {
    public:
        void setNumberOfVariables(int n) { n_ = n; }
        void setNumberOfConstraints(int m) { m_ = m; }
        bool setHessianMatrix(const Matrix &H);
        bool setGradient(const Vector &q);
        bool setLinearConstraintsMatrix(const Matrix &A);
        bool setLowerBound(const Vector &l);
        bool setUpperBound(const Vector &u);
        int n_ = -1, m_ = -1;
        Matrix P_, A_;
        Vector q_, l_, u_;
        bool hasP_ = false, hasQ_ = false, hasA_ = false, hasL_ = false, hasU_ = false;
    };

    explicit Solver(int device = 0) : device_(device) {}
    ~Solver();
    Solver(const Solver &) = delete;
    Solver &operator=(const Solver &) = delete;

    Settings *settings() { return &settings_; }
    Data *data() { return &data_; }
    bool initSolver();                  // osqp_setup (device)
    bool isInitialized() const { return ctx_ != nullptr; }
    void clearSolver();
    bool updateGradient(const Vector &q);       // osqp_update_lin_cost
    bool updateUpperBound(const Vector &u);      // osqp_update_upper_bound
    bool updateLowerBound(const Vector &l);
    bool updateBounds(const Vector &l, const Vector &u);
    bool solve();                               // osqp_solve; true iff OSQP_SOLVED
    const Vector &getSolution() const { return x_; }
    const Vector &getDualSolution() const { return y_; }
    int getStatus() const { return status_; }
    int getIterations() const { return iter_; }
    double getRho() const { return rho_; }
    const std::string &lastError() const { return err_; }

private:
    bool fail(const char *where);
    int device_;
    Settings settings_;
    Data data_;
    mpcq_ctx *ctx_ = nullptr;
    Vector x_, y_, E_, l_scaled_;
    int status_ = MPCQ_UNSOLVED, iter_ = 0;
    double rho_ = 0.0;
    std::string err_;
};

}  // namespace mpcq
