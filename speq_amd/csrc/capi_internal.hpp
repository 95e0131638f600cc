// Shared helpers for the C ABI translation units: exception -> status code + thread-local message.
#pragma once
#include <new>
#include <string>

#include "fm_index.hpp"
#include "speq_errors.hpp"
#include "speq_scan.h"

struct speq_index {
    speq::FmIndex fm;
};

namespace speq {

void set_last_error(const std::string& msg);

template <typename F>
int guarded(F&& f) {
    try {
        f();
        set_last_error("");
        return SPEQ_OK;
    } catch (const GroupsError& e) {
        set_last_error(e.what());
        return SPEQ_E_GROUPS;
    } catch (const IoError& e) {
        set_last_error(e.what());
        return SPEQ_E_IO;
    } catch (const DeviceError& e) {
        set_last_error(e.what());
        return SPEQ_E_DEVICE;
    } catch (const RetryError& e) {
        set_last_error(e.what());
        return SPEQ_E_RETRY;
    } catch (const std::bad_alloc&) {
        set_last_error("out of host memory");
        return SPEQ_E_NOMEM;
    } catch (const std::invalid_argument& e) {
        set_last_error(e.what());
        return SPEQ_E_ARG;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return SPEQ_E_ARG;
    }
}

}  // namespace speq
