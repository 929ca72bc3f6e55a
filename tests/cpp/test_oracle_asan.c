/* ASan/UBSan driver for the oracle (host code only; no GPU): the README
 * scenario KAT, and the SoA form against the reference-shaped names form on
 * random clusters, under -fsanitize=address,undefined. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/ms_oracle.h"

static unsigned long long s = 88172645463325252ull;
static unsigned rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (unsigned)s; }

int main(void) {
    int fails = 0;
    /* README scenario: node0..node8 unschedulable, then node10 */
    uint8_t flags[10] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 0}, digit[10] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 0};
    uint32_t pord = 1; int8_t pdig = 1; uint8_t ptol = 0;
    msor_nodes nd = {9, flags, digit, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL};
    msor_pods pd = {1, &pord, &pdig, &ptol, NULL, NULL, NULL, NULL};
    int32_t node, code; int64_t score; uint32_t mask; uint64_t key;
    msor_schedule(&nd, &pd, 0, 0, 1, 0, &node, &score, &code, &mask, &key);
    if (!(code == 2 && mask == 1)) { printf("README before node10 wrong\n"); ++fails; }
    nd.n = 10;
    msor_schedule(&nd, &pd, 0, 0, 1, 0, &node, &score, &code, &mask, &key);
    if (!(code == 0 && node == 9 && score == 0)) { printf("README after node10 wrong\n"); ++fails; }
    /* SoA vs names form */
    for (int trial = 0; trial < 20; ++trial) {
        uint32_t n = 1 + rnd() % 300, p = 1 + rnd() % 100;
        char **nn = calloc(n, sizeof(char *)), **pn = calloc(p, sizeof(char *));
        uint8_t *nf = calloc(n, 1), *nd8 = calloc(n, 1), *pt = calloc(p, 1);
        int8_t *pdg = calloc(p, 1); uint32_t *po = calloc(p, 4);
        int32_t *a_node = calloc(p, 4), *a_code = calloc(p, 4), *b_node = calloc(p, 4), *b_code = calloc(p, 4);
        int64_t *a_score = calloc(p, 8), *b_score = calloc(p, 8); uint32_t *a_mask = calloc(p, 4), *b_mask = calloc(p, 4);
        uint64_t *a_key = calloc(p, 8);
        for (uint32_t i = 0; i < n; ++i) {
            nn[i] = malloc(24);
            if (rnd() % 10) { snprintf(nn[i], 24, "node%u", i); nd8[i] = i % 10; }
            else { snprintf(nn[i], 24, "node-%c", 'a' + i % 26); nd8[i] = 0xFF; }
            nf[i] = (rnd() % 4 == 0) ? 1 : 0;
        }
        for (uint32_t j = 0; j < p; ++j) {
            pn[j] = malloc(24);
            if (rnd() % 10) { snprintf(pn[j], 24, "pod%u", j); pdg[j] = j % 10; }
            else { snprintf(pn[j], 24, "pod-%c", 'a' + j % 26); pdg[j] = -1; }
            pt[j] = rnd() % 5 == 0; po[j] = rnd();
        }
        msor_nodes n2 = {n, nf, nd8, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL};
        msor_pods p2 = {p, po, pdg, pt, NULL, NULL, NULL, NULL};
        msor_schedule(&n2, &p2, 0, 0, 7, 0, a_node, a_score, a_code, a_mask, a_key);
        msor_schedule_nunn_names((const char *const *)nn, nf, n, (const char *const *)pn, pt, po, p, 7, b_node, b_score, b_code, b_mask);
        for (uint32_t j = 0; j < p; ++j)
            if (a_node[j] != b_node[j] || a_code[j] != b_code[j] || a_score[j] != b_score[j] || a_mask[j] != b_mask[j]) { ++fails; printf("mismatch trial %d pod %u\n", trial, j); break; }
        for (uint32_t i = 0; i < n; ++i) free(nn[i]);
        for (uint32_t j = 0; j < p; ++j) free(pn[j]);
        free(nn); free(pn); free(nf); free(nd8); free(pt); free(pdg); free(po);
        free(a_node); free(a_code); free(b_node); free(b_code); free(a_score); free(b_score); free(a_mask); free(b_mask); free(a_key);
    }
    printf("%s\n", fails ? "FAIL" : "ok");
    return fails != 0;
}
