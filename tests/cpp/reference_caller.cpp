// tests/cpp/reference_caller.cpp — a caller written in the call shapes of LukeSchmitt96/solveMPC's
// ModelPredictiveControlAPI (src/ModelPredictiveControlAPI.cpp:42-64 setup, :81-108 controllerStep),
// with the reference's Eigen member types (include/ModelPredictiveControlAPI.h:148-200), compiled
// against include/OsqpEigen/OsqpEigen.h and the caller's own Eigen.  Test program, not product code.
//
// Input (whitespace-separated numbers, from the test): steps, then the condensed operators of the
// reference controller at mpcWindow = 15 — P (N x N), A (2N x N), Fx (N x 4), Fu (N), Fr (N x N),
// Sbar (2N x 4), Ku (2N), W0 (2N), row-major — then xref, U0 and `steps` states X (4 each).
// Output: one line per controllerStep, "U status iterations" (U printed %.17g).
// Exit: 0 ok; 3 initSolver() false (e.g. no gfx950 device); 4 controllerStep false; 2 bad input.
#include <cfloat>
#include <cstdio>
#include <fstream>
#include <limits>

#include <OsqpEigen/OsqpEigen.h>

const int mpcWindow = 15;
const int N_S = 4, N_C = 1, N_O = 1;

struct Caller {
    Eigen::SparseMatrix<double> H, Gbar;
    Eigen::Matrix<double, N_C * mpcWindow, N_S> Fx;
    Eigen::Matrix<double, N_C * mpcWindow, N_C> Fu;
    Eigen::Matrix<double, N_C * mpcWindow, N_C * mpcWindow> Fr;
    Eigen::Matrix<double, 2 * mpcWindow, 4> Sbar;
    Eigen::Matrix<double, 2 * mpcWindow, N_O> Ku;
    Eigen::Matrix<double, 2 * mpcWindow, 1> W0, lb, ub;
    Eigen::Matrix<double, N_C * mpcWindow, 1> f;
    Eigen::Matrix<double, N_S, 1> X;
    Eigen::Matrix<double, N_O, N_O> U;
    Eigen::Matrix<double, N_O, mpcWindow> ref;
    double xref = 0.0;
    OsqpEigen::Solver solver;
    bool solverFlag = true;

    void setF() { f = Fx * X + Fu * U + Fr * ref.transpose(); }  // :374

    void init(bool verbose)  // :42-64
    {
        ref = xref * Eigen::Matrix<double, N_C, mpcWindow>::Ones();
        setF();
        lb = Eigen::Matrix<double, 2 * mpcWindow, 1>::Ones() * -std::numeric_limits<double>::max();
        ub = W0 + Sbar * X + Ku * U;
        solver.settings()->setVerbosity(verbose);
        solver.settings()->setWarmStart(true);
        solver.data()->setNumberOfVariables(N_O * mpcWindow);
        solver.data()->setNumberOfConstraints(2 * mpcWindow);
        if (!solver.data()->setHessianMatrix(H))              { solverFlag = false; return; }
        if (!solver.data()->setGradient(f))                   { solverFlag = false; return; }
        if (!solver.data()->setLinearConstraintsMatrix(Gbar)) { solverFlag = false; return; }
        if (!solver.data()->setLowerBound(lb))                { solverFlag = false; return; }
        if (!solver.data()->setUpperBound(ub))                { solverFlag = false; return; }
        if (!solver.initSolver())                             { solverFlag = false; return; }
    }

    bool controllerStep()  // :81-108
    {
        ref = xref * Eigen::Matrix<double, N_C, mpcWindow>::Ones();
        setF();
        if (!solver.updateGradient(f)) return false;
        if (!solver.updateUpperBound(W0 + Sbar * X + Ku * U)) return false;
        if (!solver.solve()) return false;
        U += solver.getSolution().block<N_C, 1>(0, 0);
        return true;
    }
};

template <typename M>
static bool read_dense(std::istream &in, M &m)
{
    for (int i = 0; i < m.rows(); i++)
        for (int j = 0; j < m.cols(); j++)
            if (!(in >> m(i, j))) return false;
    return true;
}

static bool read_sparse(std::istream &in, Eigen::SparseMatrix<double> &S, int rows, int cols)
{
    S.resize(rows, cols);
    for (int i = 0; i < rows; i++)
        for (int j = 0; j < cols; j++) {
            double v;
            if (!(in >> v)) return false;
            S.insert(i, j) = v;  // every entry, explicit zeros included (:254-263, :339-347)
        }
    S.makeCompressed();
    return true;
}

int main(int argc, char **argv)
{
    if (argc < 2) return 2;
    std::ifstream in(argv[1]);
    const bool verbose = argc > 2;
    int steps = 0;
    Caller c;
    if (!(in >> steps) || !read_sparse(in, c.H, mpcWindow, mpcWindow) || !read_sparse(in, c.Gbar, 2 * mpcWindow, mpcWindow) ||
        !read_dense(in, c.Fx) || !read_dense(in, c.Fu) || !read_dense(in, c.Fr) || !read_dense(in, c.Sbar) ||
        !read_dense(in, c.Ku) || !read_dense(in, c.W0) || !(in >> c.xref) || !(in >> c.U(0)))
        return 2;
    c.X.setZero();
    c.init(verbose);
    if (!c.solverFlag) {
        std::printf("initSolver failed: %s\n", c.solver.lastError().c_str());
        return 3;
    }
    for (int k = 0; k < steps; k++) {
        if (!read_dense(in, c.X)) return 2;
        if (!c.controllerStep()) {
            std::printf("controllerStep failed at step %d: status %d\n", k, c.solver.getStatus());
            return 4;
        }
        std::printf("%.17g %d %d\n", c.U(0), c.solver.getStatus(), c.solver.getIterations());
    }
    return 0;
}
