/* A C99 caller of include/gnark_amd.h, shaped like the cgo shim
 * (go/backend/groth16/bn254/amd/amd.go; the reference's icicle.go:133-422 and
 * groth16_test.go:70-88): upload the proving key once with
 * gg_groth16_pk_create, prove with gg_groth16_prove from host buffers, print
 * the proof.  Built by tests/test_c_caller.py with
 *     gcc -std=c99 -pedantic -Wall -Werror -I include ... -lgnark_amd
 * which is what cgo does with the header.
 *
 * Input (stdin): lines "name hex" for log_n, nb_public, omega, coset_gen, g1_A,
 * g1_B, g1_Z, g1_K, alpha1, beta1, delta1, g2_B, beta2, delta2, infA, infB,
 * wires, solA, solB, solC, r, s (small integers as decimal).  Output (stdout):
 * "Ar <hex>", "Bs <hex>", "Krs <hex>", or "ERR <code> <message>" and exit 1. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gnark_amd.h"

#define MAX_FIELDS 32

struct field {
    char name[32];
    unsigned char *data;
    size_t len;
    long value;
};

static struct field fields[MAX_FIELDS];
static int nfields = 0;

static int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static const struct field *get(const char *name) {
    int i;
    for (i = 0; i < nfields; i++)
        if (strcmp(fields[i].name, name) == 0) return &fields[i];
    fprintf(stdout, "ERR -1 missing input %s\n", name);
    exit(1);
    return NULL;
}

static void read_input(void) {
    static char line[1 << 20];
    while (fgets(line, sizeof line, stdin)) {
        char *sp = strchr(line, ' ');
        struct field *f;
        size_t n, i;
        char *v;
        if (!sp || nfields == MAX_FIELDS) continue;
        *sp = 0;
        v = sp + 1;
        n = strcspn(v, "\r\n");
        v[n] = 0;
        f = &fields[nfields++];
        strncpy(f->name, line, sizeof f->name - 1);
        f->value = strtol(v, NULL, 10);
        f->len = n / 2;
        f->data = (unsigned char *)malloc(f->len ? f->len : 1);
        for (i = 0; i < f->len; i++) f->data[i] = (unsigned char)(hexval(v[2 * i]) * 16 + hexval(v[2 * i + 1]));
    }
}

static void put_hex(const char *name, const unsigned char *p, size_t n) {
    size_t i;
    printf("%s ", name);
    for (i = 0; i < n; i++) printf("%02x", p[i]);
    printf("\n");
}

static int fail(int rc) {
    printf("ERR %d %s\n", rc, gg_last_error());
    return 1;
}

int main(void) {
    gg_groth16_pk_t pk = NULL;
    unsigned char ar[64], bs[128], krs[64];
    const struct field *g1_A, *g1_B, *g1_Z, *g1_K, *g2_B, *infA, *wires, *solA;
    int log_n, rc;
    size_t n_wires, n_cons;
    read_input();
    log_n = (int)get("log_n")->value;
    g1_A = get("g1_A");
    g1_B = get("g1_B");
    g1_Z = get("g1_Z");
    g1_K = get("g1_K");
    g2_B = get("g2_B");
    infA = get("infA");
    wires = get("wires");
    solA = get("solA");
    n_wires = infA->len;
    n_cons = solA->len / 32;
    if (wires->len != 32 * n_wires) {
        printf("ERR -1 wire vector of %lu bytes for %lu wires\n", (unsigned long)wires->len, (unsigned long)n_wires);
        return 1;
    }
    rc = gg_groth16_pk_create(log_n, get("omega")->data, get("coset_gen")->data, g1_A->data, g1_A->len / 64,
                              g1_B->data, g1_B->len / 64, g1_Z->data, g1_Z->len / 64, g1_K->data, g1_K->len / 64,
                              get("alpha1")->data, get("beta1")->data, get("delta1")->data, g2_B->data,
                              get("beta2")->data, get("delta2")->data, infA->data, get("infB")->data, n_wires,
                              (size_t)get("nb_public")->value, NULL, &pk);
    if (rc != GG_OK) return fail(rc);
    /* gnark proves many times with one key (the shim caches it): prove twice */
    rc = gg_groth16_prove(pk, wires->data, n_wires, solA->data, get("solB")->data, get("solC")->data, n_cons, 0,
                          get("r")->data, get("s")->data, ar, bs, krs, NULL);
    if (rc == GG_OK)
        rc = gg_groth16_prove(pk, wires->data, n_wires, solA->data, get("solB")->data, get("solC")->data, n_cons,
                              0, get("r")->data, get("s")->data, ar, bs, krs, NULL);
    if (rc != GG_OK) {
        gg_groth16_pk_release(pk);
        return fail(rc);
    }
    put_hex("Ar", ar, sizeof ar);
    put_hex("Bs", bs, sizeof bs);
    put_hex("Krs", krs, sizeof krs);
    rc = gg_groth16_pk_release(pk);
    if (rc != GG_OK) return fail(rc);
    return 0;
}
