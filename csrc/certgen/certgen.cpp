// Self-signed serving certificate for the supervisor's shard-label admission webhook
// (nexus_supervisor_amd/webhook_certs.py; sharding.webhook-cert-bootstrap).
//
// The API server only calls HTTPS webhooks and verifies them against the
// MutatingWebhookConfiguration's caBundle.  Without cert-manager the replicas mint the
// pair themselves: a CA (P-256, CA:TRUE, keyCertSign) and a serving certificate for the
// webhook Service's DNS names signed by it (serverAuth, SAN DNS entries).  Python's ssl
// module cannot create certificates and the `cryptography` package is not part of the
// image, so this is libcrypto (OpenSSL 3) directly; no counterpart in the reference,
// which has no webhook.
#include <openssl/bio.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rand.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct PkeyDel {
  void operator()(EVP_PKEY* p) const { EVP_PKEY_free(p); }
};
struct X509Del {
  void operator()(X509* x) const { X509_free(x); }
};
struct BioDel {
  void operator()(BIO* b) const { BIO_free(b); }
};
using Pkey = std::unique_ptr<EVP_PKEY, PkeyDel>;
using Cert = std::unique_ptr<X509, X509Del>;
using Bio = std::unique_ptr<BIO, BioDel>;

[[noreturn]] void fail(const char* what) { throw std::runtime_error(std::string("certgen: ") + what); }

Pkey ec_key() {
  EVP_PKEY* k = EVP_EC_gen("P-256");
  if (!k) fail("EC key generation failed");
  return Pkey(k);
}

void add_ext(X509* cert, X509* issuer, int nid, const std::string& value) {
  X509V3_CTX ctx;
  X509V3_set_ctx_nodb(&ctx);
  X509V3_set_ctx(&ctx, issuer, cert, nullptr, nullptr, 0);
  X509_EXTENSION* ext = X509V3_EXT_conf_nid(nullptr, &ctx, nid, value.c_str());
  if (!ext) fail("bad extension");
  int ok = X509_add_ext(cert, ext, -1);
  X509_EXTENSION_free(ext);
  if (!ok) fail("X509_add_ext");
}

Cert new_cert(EVP_PKEY* key, const std::string& cn, long days, long backdate_s) {
  Cert x(X509_new());
  if (!x) fail("X509_new");
  X509_set_version(x.get(), 2);  // v3
  unsigned char serial[16];
  if (RAND_bytes(serial, sizeof serial) != 1) fail("RAND_bytes");
  serial[0] &= 0x7f;  // positive
  BIGNUM* bn = BN_bin2bn(serial, sizeof serial, nullptr);
  if (!bn || !BN_to_ASN1_INTEGER(bn, X509_get_serialNumber(x.get()))) fail("serial");
  BN_free(bn);
  X509_gmtime_adj(X509_getm_notBefore(x.get()), -backdate_s);  // tolerate clock skew
  X509_gmtime_adj(X509_getm_notAfter(x.get()), days * 86400L);
  if (!X509_set_pubkey(x.get(), key)) fail("X509_set_pubkey");
  X509_NAME* name = X509_get_subject_name(x.get());
  X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_UTF8, reinterpret_cast<const unsigned char*>(cn.c_str()), -1, -1, 0);
  return x;
}

std::string pem_cert(X509* x) {
  Bio b(BIO_new(BIO_s_mem()));
  if (!b || !PEM_write_bio_X509(b.get(), x)) fail("PEM_write_bio_X509");
  char* data = nullptr;
  long n = BIO_get_mem_data(b.get(), &data);
  return std::string(data, static_cast<size_t>(n));
}

std::string pem_key(EVP_PKEY* k) {
  Bio b(BIO_new(BIO_s_mem()));
  if (!b || !PEM_write_bio_PrivateKey(b.get(), k, nullptr, nullptr, 0, nullptr, nullptr)) fail("PEM_write_bio_PrivateKey");
  char* data = nullptr;
  long n = BIO_get_mem_data(b.get(), &data);
  return std::string(data, static_cast<size_t>(n));
}

// (ca_pem, cert_pem, key_pem): a fresh CA and a serving certificate for `dns_names`
// (the first is the subject CN) valid `days` days.
py::tuple mint(const std::string& ca_name, const std::vector<std::string>& dns_names, long days) {
  if (dns_names.empty()) fail("at least one DNS name is required");
  if (days < 1 || days > 3650) fail("days must be in [1, 3650]");
  std::string ca_pem, cert_pem, key_pem;
  {
    py::gil_scoped_release nogil;
    Pkey ca_key = ec_key();
    Cert ca = new_cert(ca_key.get(), ca_name, days + 1, 300);
    X509_set_issuer_name(ca.get(), X509_get_subject_name(ca.get()));
    add_ext(ca.get(), ca.get(), NID_basic_constraints, "critical,CA:TRUE,pathlen:0");
    add_ext(ca.get(), ca.get(), NID_key_usage, "critical,keyCertSign,cRLSign");
    add_ext(ca.get(), ca.get(), NID_subject_key_identifier, "hash");
    if (!X509_sign(ca.get(), ca_key.get(), EVP_sha256())) fail("signing the CA");

    Pkey key = ec_key();
    Cert leaf = new_cert(key.get(), dns_names[0], days, 300);
    X509_set_issuer_name(leaf.get(), X509_get_subject_name(ca.get()));
    std::string san;
    for (const auto& d : dns_names) san += (san.empty() ? "DNS:" : ",DNS:") + d;
    add_ext(leaf.get(), ca.get(), NID_basic_constraints, "critical,CA:FALSE");
    add_ext(leaf.get(), ca.get(), NID_key_usage, "critical,digitalSignature,keyEncipherment");
    add_ext(leaf.get(), ca.get(), NID_ext_key_usage, "serverAuth");
    add_ext(leaf.get(), ca.get(), NID_subject_alt_name, san);
    add_ext(leaf.get(), ca.get(), NID_subject_key_identifier, "hash");
    add_ext(leaf.get(), ca.get(), NID_authority_key_identifier, "keyid:always");
    if (!X509_sign(leaf.get(), ca_key.get(), EVP_sha256())) fail("signing the serving certificate");
    ca_pem = pem_cert(ca.get());
    cert_pem = pem_cert(leaf.get());
    key_pem = pem_key(key.get());
  }
  return py::make_tuple(ca_pem, cert_pem, key_pem);
}

}  // namespace

PYBIND11_MODULE(_certgen, m) {
  m.doc() = "Self-signed CA + serving certificate for the shard-label webhook (libcrypto)";
  m.def("mint", &mint, py::arg("ca_name"), py::arg("dns_names"), py::arg("days") = 365,
        "(ca_pem, cert_pem, key_pem): a P-256 CA and a serverAuth certificate for dns_names signed by it");
}
