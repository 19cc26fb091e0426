// host_pool.h -- a fixed pool of host threads with a FIFO of tasks (the batch's
// host coders; the band-parallel modelling of one plane's encode).
#pragma once
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ric {

// A fixed pool of host coder threads with a FIFO of tasks.
class Pool {
public:
	explicit Pool(int n)
	{
		for (int i = 0; i < n; i++) th_.emplace_back([this] { run(); });
	}
	~Pool()
	{
		{
			std::lock_guard<std::mutex> g(mu_);
			stop_ = true;
		}
		cv_.notify_all();
		for (auto& t : th_) t.join();
	}
	void submit(std::function<void()> f)
	{
		{
			std::lock_guard<std::mutex> g(mu_);
			q_.push_back(std::move(f));
		}
		cv_.notify_one();
	}
	int size() const { return (int)th_.size(); }

private:
	void run()
	{
		for (;;) {
			std::function<void()> f;
			{
				std::unique_lock<std::mutex> lk(mu_);
				cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
				if (q_.empty()) return;
				f = std::move(q_.front());
				q_.pop_front();
			}
			f();
		}
	}
	std::vector<std::thread> th_;
	std::deque<std::function<void()>> q_;
	std::mutex mu_;
	std::condition_variable cv_;
	bool stop_ = false;
};

}  // namespace ric
