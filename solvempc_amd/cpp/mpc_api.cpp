// solvempc_amd/cpp/mpc_api.cpp — ModelPredictiveControlAPI on MI355X (see mpc_api.hpp).
#include "mpc_api.hpp"

#include <algorithm>
#include <cfloat>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>

using mpcq::Matrix;

namespace {
// "<name> rows: r\t<name> cols: c" / "<name>:" / matrix / blank line, as the reference's -v dumps
// print every operator (ModelPredictiveControlAPI.cpp:122-132 and the other set* builders).
void dump(const char *name, const Matrix &m, const char *cols_name = nullptr)
{
    std::cout << name << " rows: " << m.rows() << "\t" << (cols_name ? cols_name : name) << " cols: " << m.cols()
              << std::endl;
    std::cout << name << ":" << std::endl << m << std::endl << std::endl;
}

Matrix matpow(const Matrix &A, int k)
{
    Matrix r(A.rows(), A.cols());
    for (int i = 0; i < A.rows(); i++) r(i, i) = 1.0;
    for (int t = 0; t < k; t++) r = r * A;
    return r;
}
}  // namespace

ModelPredictiveControlAPI::ModelPredictiveControlAPI(bool verbose_, const std::string &config, int N, int device)
    : solver(device), horizon(N), device_(device)
{
    std::cout << "[MPC API]\tMPC API object created." << std::endl;
    verbose = verbose_;
    solverFlag = true;
    std::ifstream file(config);  // CWD-relative by default, like the reference (:12)
    if (!file)  // json::parse of an unopened stream sees an empty input (:13)
        throw json_lite::detail::parse_error::create(101, 1, "syntax error while parsing value - unexpected end of input (" + config + ")");
    std::stringstream ss;
    ss << file.rdbuf();
    cfg = json_lite::parse(ss.str());
    K = from_json(cfg["K"], 1, N_S);
    xref = cfg["xref"].get_double();
    X = Matrix::Zero(N_S, 1);
    U = Matrix::Zero(N_O, N_O);
    t0 = dt = 0.0;

    // The condensing runs on the device (condense_on_device).  A host without a usable MI355X fails here:
    // that is this drop-in's counterpart of the reference's solver failure, so it takes the same exit,
    // solverFlag = false (the caller's `if(!mpc.solverFlag){return 1;}`, solver.cpp:28), with the
    // library's reason on stderr, instead of an exception the reference's caller does not catch.
    try {
        setSystemVars();
        setCosts();
        setLiftedCosts();
        setTransformations();
        setLL();
        setH();
        setLu();
        setFVars();
        setLinearConstraints();
        setUpperBound();
        updateRef(xref);
        setF();
    } catch (const DeviceError &e) {
        std::cerr << e.what() << std::endl;
        solverFlag = false;
        return;
    }

    lb = Matrix(2 * horizon, 1, -DBL_MAX);  // :42
    ub = Matrix(2 * horizon, 1);            // :43  W0 + Sbar X + Ku U
    for (int i = 0; i < 2 * horizon; i++) {
        double s = 0.0;
        for (int c = 0; c < N_S; c++) s += Sbar(i, c) * X(c);
        ub(i) = W0(i) + s + Ku(i) * U(0);
    }
    std::cout << "[MPC API]\tAll QP matrices built successfully." << std::endl;

    n_variables = N_O * horizon;
    n_constraints = 2 * horizon;
    solver.settings()->setVerbosity(verbose);
    solver.settings()->setWarmStart(true);
    solver.data()->setNumberOfVariables(n_variables);
    solver.data()->setNumberOfConstraints(n_constraints);
    if (!solver.data()->setHessianMatrix(H)) { solverFlag = false; return; }
    if (!solver.data()->setGradient(std::vector<double>(f.data(), f.data() + f.size()))) { solverFlag = false; return; }
    if (!solver.data()->setLinearConstraintsMatrix(Gbar)) { solverFlag = false; return; }
    if (!solver.data()->setLowerBound(std::vector<double>(lb.data(), lb.data() + lb.size()))) { solverFlag = false; return; }
    if (!solver.data()->setUpperBound(std::vector<double>(ub.data(), ub.data() + ub.size()))) { solverFlag = false; return; }
    if (!solver.initSolver()) { solverFlag = false; return; }
}

ModelPredictiveControlAPI::~ModelPredictiveControlAPI()
{
    std::printf("[MPC API]\tDestructing MPC API object...\n");
}

void ModelPredictiveControlAPI::setVerbosity(bool v)
{
    verbose = v;
    std::cout << "[MPC API]\tVerbosity set to " << verbose << std::endl;
}

void ModelPredictiveControlAPI::setSystemVars()
{
    Ad = from_json(cfg["Ad"], N_S, N_S);
    Bd = from_json(cfg["Bd"], N_S, N_C);
    Cd = from_json(cfg["Cd"], N_O, N_S);
    Dd = from_json(cfg["Dd"], N_O, N_C);
    if (verbose) {
        std::cout << "[MPC API]\tSystem variables created." << std::endl;
        dump("Ad", Ad);
        dump("Bd", Bd);
        dump("Cd", Cd);
        dump("Dd", Dd);
    }
}

void ModelPredictiveControlAPI::setCosts()
{
    Q = from_json(cfg["Q"], N_O, N_O);
    R = from_json(cfg["R"], N_O, N_O);
    RD = from_json(cfg["RD"], N_O, N_O);
    if (verbose) {
        std::cout << "[MPC API]\tSet Q, R, and RD matrices created." << std::endl;
        dump("Q", Q);
        dump("R", R);
        dump("RD", RD);
    }
}

void ModelPredictiveControlAPI::setLiftedCosts()
{
    Qbar = blkdiag(Q, horizon);
    Rbar = blkdiag(R, horizon);
    RbarD = blkdiag(RD, horizon);
    if (verbose) {
        std::cout << "[MPC API]\tLifted weight matrices created." << std::endl;
        dump("Qbar", Qbar);
        dump("Rbar", Rbar);
        dump("RbarD", RbarD);
    }
}

// The condensed operators come from the device kernel (mpcq_condense), built once here and
// handed out by the individual set* builders below.
void ModelPredictiveControlAPI::condense_on_device()
{
    const int N = horizon;
    std::vector<double> P(N * N), A(2 * N * N), fx(N * N_S), fu(N), fr(N * N), sbar(2 * N * N_S), ku(2 * N), w0(2 * N);
    const std::vector<double> ad = Ad.row_major(), bd = Bd.row_major(), cd = Cd.row_major(), k = K.row_major();
    const double q = Q(0, 0), r = R(0, 0), rd = RD(0, 0);
    if (mpcq_condense(device_, 1, N_S, N, 10, ad.data(), bd.data(), cd.data(), k.data(), &q, &r, &rd, P.data(),
                      A.data(), fx.data(), fu.data(), fr.data(), sbar.data(), ku.data(), w0.data()) != MPCQ_OK)
        throw DeviceError(std::string("[MPC API]\tcondensing failed: ") + mpcq_last_error());
    H = Matrix::from_row_major(N, N, P.data());
    Gbar = Matrix::from_row_major(2 * N, N, A.data());
    Fx = Matrix::from_row_major(N, N_S, fx.data());
    Fu = Matrix::from_row_major(N, 1, fu.data());
    Fr = Matrix::from_row_major(N, N, fr.data());
    Sbar = Matrix::from_row_major(2 * N, N_S, sbar.data());
    Ku = Matrix::from_row_major(2 * N, 1, ku.data());
    W0 = Matrix::from_row_major(2 * N, 1, w0.data());
    S = Matrix(N, N_S);
    for (int i = 0; i < N; i++)
        for (int c = 0; c < N_S; c++) S(i, c) = Sbar(i, c);
    condensed_ = true;
}

// The -v dump of setTransformations (:210-243) prints intermediate matrices the QP never reads (the
// device kernel builds every operator it does read).  They are formed here for printing only.
void ModelPredictiveControlAPI::transformations_for_dump(Matrix &CAB, Matrix &CAiB, Matrix &CAB_full,
                                                         Matrix &Su_full, Matrix &Su_full1) const
{
    const int N = horizon;
    CAB = Matrix(N, 1);
    CAiB = Matrix(N_S, N_O);
    CAB_full = Matrix(N_S * N, N_O);
    Sx = Matrix(N, N_S);
    for (int i = 0; i < N; i++) {
        const Matrix Ai = matpow(Ad, i), Ai1 = Ai * Ad;
        const Matrix cx = Cd * Ai1, cab = Cd * Ai * Bd, aib = Ai * Bd;
        for (int c = 0; c < N_S; c++) Sx(i, c) = cx(0, c);
        CAB(i) = cab(0, 0);
        for (int r = 0; r < N_S; r++) CAiB(r) += aib(r, 0);
        for (int r = 0; r < N_S; r++) CAB_full(N_S * i + r) = CAiB(r);
    }
    Su = Matrix(N, N);  // strict upper triangle never written (:197-204): zero here
    Su_full = Matrix(N_S * N, N);
    for (int i = 0; i < N; i++)
        for (int j = 0; j <= i; j++) {
            double acc = 0.0;
            for (int k = 0; k <= i - j; k++) acc += CAB(k);
            Su(i, j) = acc;
            for (int r = 0; r < N_S; r++) Su_full(N_S * i + r, j) = CAB_full(N_S * (i - j) + r);
        }
    Su1 = Matrix(N, N_O);
    Su_full1 = Matrix(N_S * N, 1);
    for (int i = 0; i < N; i++) Su1(i) = Su(i, 0);
    for (int i = 0; i < N_S * N; i++) Su_full1(i) = Su_full(i, 0);
}

void ModelPredictiveControlAPI::setTransformations()
{
    if (!condensed_) condense_on_device();
    if (verbose) {
        std::cout << "[MPC API]\tTransformation matrices created" << std::endl;
        Matrix CAB, CAiB, CAB_full, Su_full, Su_full1;
        transformations_for_dump(CAB, CAiB, CAB_full, Su_full, Su_full1);
        dump("Sx", Sx);
        dump("CAB", CAB);
        dump("CAiB", CAiB);
        dump("CAB_full", CAB_full);
        dump("S", S);
        dump("Su", Su);
        dump("Su1", Su1);
        dump("Su_full", Su_full, "Su1");  // (the reference labels these columns "Su1", :235,238)
        dump("Su_full1", Su_full1, "Su1");
        dump("Sbar", Sbar);
    }
}

void ModelPredictiveControlAPI::setH()
{
    if (!condensed_) condense_on_device();
    if (verbose) {
        std::cout << "[MPC API]\tHessian H created." << std::endl;
        dump("H", H);
    }
}

void ModelPredictiveControlAPI::setLu()
{
    Lu = Matrix(horizon, 1);  // (mpcWindow - i + 2), unused by the QP (:274-279)
    for (int i = 0; i < horizon; i++) Lu(i) = horizon - i + 2;
    if (verbose) {
        std::cout << "[MPC API]\tLu created." << std::endl;
        dump("Lu", Lu);
    }
}

void ModelPredictiveControlAPI::setLL()
{
    LL = Matrix(horizon, horizon);
    for (int i = 0; i < horizon; i++)
        for (int j = 0; j <= i; j++) LL(i, j) = 1.0;
    if (verbose) {
        std::cout << "[MPC API]\tLL created." << std::endl;
        dump("LL", LL);
    }
}

void ModelPredictiveControlAPI::setFVars()
{
    if (!condensed_) condense_on_device();
    if (verbose) {
        std::cout << "[MPC API]\tComponents of F created." << std::endl;
        dump("Fu", Fu);
        dump("Fr", Fr);
        dump("Fx", Fx);
    }
}

void ModelPredictiveControlAPI::setLinearConstraints()
{
    if (!condensed_) condense_on_device();
    if (verbose) {
        std::cout << "[MPC API]\tLinear constraints matrix created." << std::endl;
        dump("Gbar", Gbar);
    }
}

void ModelPredictiveControlAPI::setUpperBound()
{
    // Ku = [-K0 1; K0 1], W0 = 255 1 (:364-368) — constants, already on the condensed result
    if (!condensed_) condense_on_device();
}

void ModelPredictiveControlAPI::setF()
{
    // f = Fx X + Fu U + Fr ref'  (:374)
    f = Matrix(horizon, 1);
    for (int i = 0; i < horizon; i++) {
        double a = 0.0, c = 0.0;
        for (int t = 0; t < N_S; t++) a += Fx(i, t) * X(t);
        const double b = Fu(i) * U(0);
        for (int t = 0; t < horizon; t++) c += Fr(i, t) * ref(t);
        f(i) = a + b + c;
    }
}

void ModelPredictiveControlAPI::updateRef(double pos_ref)
{
    ref = Matrix(1, horizon, pos_ref);
    if (verbose) std::cout << "[MPC API]\tref: " << ref << std::endl;
}

bool ModelPredictiveControlAPI::controllerStep()
{
    t0 += dt;
    updateRef(xref);
    setF();
    setUpperBound();
    if (!solver.updateGradient(std::vector<double>(f.data(), f.data() + f.size()))) return false;
    std::vector<double> u(2 * horizon);
    for (int i = 0; i < 2 * horizon; i++) {
        double s = 0.0;
        for (int c = 0; c < N_S; c++) s += Sbar(i, c) * X(c);
        u[i] = W0(i) + s + Ku(i) * U(0);
    }
    if (!solver.updateUpperBound(u)) return false;
    if (!solver.solve()) return false;
    U(0) += solver.getSolution()[0];  // receding horizon (:105)
    return true;
}

Matrix ModelPredictiveControlAPI::blkdiag(const Matrix &a, int count)
{
    Matrix b(a.rows() * count, a.cols() * count);
    for (int i = 0; i < count; i++)
        for (int r = 0; r < a.rows(); r++)
            for (int c = 0; c < a.cols(); c++) b(i * a.rows() + r, i * a.cols() + c) = a(r, c);
    return b;
}

// from_json (:418-489): a scalar, a row or column vector, or a matrix (array of rows), shape-checked
// against (rows, cols); every failure prints the reference's stderr line where it has one and throws
// json_lite's type_error::create(0, "") as the reference throws nlohmann's.  Element conversion
// follows json's: a non-number element throws type_error 302, a scalar row indexed as an array 304.
Matrix ModelPredictiveControlAPI::from_json(const json_lite::Value &jsonObject, int rows, int cols)
{
    using json_lite::Value;
    using json_lite::detail::type_error;
    Value jsonArray;
    jsonArray.kind = Value::Array;
    if (jsonObject.is_array()) {
        if (jsonObject.empty()) return Matrix(rows, cols);  // (:425-428; Eigen leaves it uninitialised)
        jsonArray = jsonObject;
    } else if (jsonObject.is_number()) {
        jsonArray.arr.push_back(jsonObject);
    } else {
        throw type_error::create(0, "");  // (:437)
    }
    Value aoa;
    aoa.kind = Value::Array;
    if (jsonArray.arr.front().is_array()) {
        aoa = jsonArray;  // provided matrix
    } else if (rows == 1) {
        aoa.arr.push_back(jsonArray);  // row vector
    } else if (cols == 1) {
        for (const Value &v : jsonArray.arr) {  // column vector
            Value row;
            row.kind = Value::Array;
            row.arr.push_back(v);
            aoa.arr.push_back(row);
        }
    } else {
        std::cerr << "Expected a matrix, received a vector." << std::endl;
        throw type_error::create(0, "");  // (:460-461)
    }
    const int pr = (int)aoa.size(), pc = (int)aoa.arr.front().size();
    if ((rows >= 0 && pr != rows) || (cols >= 0 && pc != cols)) {
        std::cerr << "Expected matrix of size " << rows << "x" << cols << ", received matrix of size " << pr << "x" << pc
                  << "." << std::endl;
        throw type_error::create(0, "");  // (:471)
    }
    Matrix m(pr, pc);
    for (int r = 0; r < pr; r++) {
        if ((int)aoa.at(r).size() != pc) {
            std::cerr << "Unconsistent matrix size: some rows have different number of columns." << std::endl;
            throw type_error::create(0, "");  // (:480)
        }
        for (int c = 0; c < pc; c++) m(r, c) = aoa.at(r).at(c).get_double();
    }
    return m;
}

char *getCmdOption(char **begin, char **end, const std::string &option)
{
    char **itr = std::find(begin, end, option);
    if (itr != end && ++itr != end) return *itr;
    return nullptr;
}

bool cmdOptionExists(char **begin, char **end, const std::string &option)
{
    return std::find(begin, end, option) != end;
}
