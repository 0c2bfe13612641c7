// bf16 library-GEMM probe for tools/tune_gemms_bf16.py (a tuning tool, not part of the product).
//
// For one GEMM as PyTorch TunableOp hands it to hipBLASLt (GemmHipblaslt.h HipblasltGemmOp::Call:
// column-major, A/B/C bf16, fp32 compute and scale, optional bf16 bias epilogue, strided batch),
// asks hipBLASLt's heuristic for its top-k solutions (NOT the full solution list TunableOp's own
// search walks: a candidate of that search faulted the GPU in round 2), and times each. Every
// candidate's solution index is printed and flushed BEFORE it runs, so a fault names its solution.
//
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/gemm_probe.cpp -lhipblaslt -o
//        tools/_bin/libgemm_probe.so (git-ignored, travels to the GPU box)
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        auto _s = (x);                                                                \
        if ((int)_s != 0) {                                                           \
            fprintf(stderr, "gemm_probe: %s failed (%d) line %d\n", #x, (int)_s, __LINE__); \
            fflush(stderr);                                                           \
            return -1;                                                                \
        }                                                                             \
    } while (0)

// transa / transb: 'n' or 't' (BLAS column-major, TunableOp's params signature); returns the number
// of candidates timed (<= topk), their solution indices and average milliseconds.
extern "C" int gemm_probe(char transa, char transb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
                          int64_t ldc, int32_t batch, int64_t stride_a, int64_t stride_b, int64_t stride_c,
                          int32_t with_bias, int32_t topk, uint64_t max_workspace, int32_t iters, int32_t* out_index,
                          float* out_ms) {
    const hipblasOperation_t opa = (transa == 'n' || transa == 'N') ? HIPBLAS_OP_N : HIPBLAS_OP_T;
    const hipblasOperation_t opb = (transb == 'n' || transb == 'N') ? HIPBLAS_OP_N : HIPBLAS_OP_T;
    const int64_t a_rows = opa == HIPBLAS_OP_N ? m : k, a_cols = opa == HIPBLAS_OP_N ? k : m;
    const int64_t b_rows = opb == HIPBLAS_OP_N ? k : n, b_cols = opb == HIPBLAS_OP_N ? n : k;
    const int64_t nb = batch > 1 ? batch : 1;
    const size_t a_elems = (size_t)(nb > 1 ? stride_a * (nb - 1) : 0) + (size_t)lda * a_cols;
    const size_t b_elems = (size_t)(nb > 1 ? stride_b * (nb - 1) : 0) + (size_t)ldb * b_cols;
    const size_t c_elems = (size_t)(nb > 1 ? stride_c * (nb - 1) : 0) + (size_t)ldc * n;
    void *A, *B, *C, *D, *bias = nullptr, *ws = nullptr;
    CK(hipMalloc(&A, a_elems * 2));
    CK(hipMalloc(&B, b_elems * 2));
    CK(hipMalloc(&C, c_elems * 2));
    CK(hipMalloc(&D, c_elems * 2));
    CK(hipMemset(A, 0x3c, a_elems * 2));  // 0x3c3c = bf16 0.0115
    CK(hipMemset(B, 0x3c, b_elems * 2));
    CK(hipMemset(C, 0, c_elems * 2));
    if (with_bias) {
        CK(hipMalloc(&bias, m * 2));
        CK(hipMemset(bias, 0, m * 2));
    }
    if (max_workspace) CK(hipMalloc(&ws, max_workspace));

    hipblasLtHandle_t handle;
    CK(hipblasLtCreate(&handle));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, a_rows, a_cols, lda));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, b_rows, b_cols, ldb));
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, m, n, ldc));
    if (batch > 1) {
        CK(hipblasLtMatrixLayoutSetAttribute(la, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &batch, sizeof(batch)));
        CK(hipblasLtMatrixLayoutSetAttribute(la, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &stride_a, 8));
        CK(hipblasLtMatrixLayoutSetAttribute(lb, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &batch, sizeof(batch)));
        CK(hipblasLtMatrixLayoutSetAttribute(lb, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &stride_b, 8));
        CK(hipblasLtMatrixLayoutSetAttribute(lc, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &batch, sizeof(batch)));
        CK(hipblasLtMatrixLayoutSetAttribute(lc, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &stride_c, 8));
    }
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
    if (with_bias) {
        const hipDataType bt = HIP_R_16BF;
        const hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    }
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &max_workspace,
                                             sizeof(max_workspace)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(topk);
    int got = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(handle, desc, la, lb, lc, lc, pref, topk, res.data(), &got));
    const float alpha = 1.0f, beta = 0.0f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int done = 0;
    for (int i = 0; i < got; ++i) {
        if (res[i].state != HIPBLAS_STATUS_SUCCESS) continue;
        const int idx = hipblaslt_ext::getIndexFromAlgo(res[i].algo);
        printf("gemm_probe: candidate %d solution %d workspace %zu\n", i, idx, (size_t)res[i].workspaceSize);
        fflush(stdout);
        for (int w = 0; w < 3; ++w)
            CK(hipblasLtMatmul(handle, desc, &alpha, A, la, B, lb, &beta, C, lc, D, lc, &res[i].algo, ws,
                               max_workspace, 0));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; ++it)
            CK(hipblasLtMatmul(handle, desc, &alpha, A, la, B, lb, &beta, C, lc, D, lc, &res[i].algo, ws,
                               max_workspace, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        out_index[done] = idx;
        out_ms[done] = ms / iters;
        printf("gemm_probe: solution %d %.4f ms\n", idx, ms / iters);
        fflush(stdout);
        ++done;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatmulDescDestroy(desc);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtDestroy(handle);
    hipFree(A);
    hipFree(B);
    hipFree(C);
    hipFree(D);
    if (bias) hipFree(bias);
    if (ws) hipFree(ws);
    return done;
}
